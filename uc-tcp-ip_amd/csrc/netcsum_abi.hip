// netcsum_abi.hip — extern "C" entry points of include/netcsum_mi355x.h groups (2) and (3):
// argument checks, launch-geometry policy, per-thread device contexts for the host-memory paths.
// Group (1) — the reference's four signatures — lives in ../host/net_util_mi355x.c (plain C) and
// reaches the GPU through NetUtil_MI355X_StreamSum32 below.
//
// There is deliberately NO CPU fallback anywhere in this library: if the HIP runtime or device
// fails, the caller gets NET_UTIL_ERR_MI355X_DEV and a message on stderr.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/netcsum_mi355x.h"
#include "netcsum_device.h"
#include "netcsum_kernels.h"

namespace {

constexpr int kMaxDev = 64;
constexpr size_t kZeroCopyMax = 16u * 1024u;      // streams up to 16 KiB: zero-copy single-block path

thread_local netcsum::TuneKnob g_tune_grid{0};
thread_local netcsum::TuneKnob g_tune_group{0};
thread_local netcsum::TuneKnob g_tune_nt{-1};                   // -1: auto (nt when groups share no chunks)
thread_local netcsum::TuneKnob g_tune_block{256};
thread_local netcsum::TuneKnob g_tune_chain_combine{-1};         // NETCSUM_TUNE_CHAIN_COMBINE
thread_local netcsum::TuneKnob g_tune_kernel{0};                 // 0 = auto (5 when small_supported, else 2)
thread_local netcsum::TuneKnob g_tune_chunks{0};
thread_local netcsum::TuneKnob g_tune_probe{1};                 // LDS-DMA read probe by default
thread_local netcsum::TuneKnob g_tune_grid_mult{1};
thread_local netcsum::TuneKnob g_tune_tile{-1};                 // -1: auto (4 segments per group per block tile)
thread_local netcsum::TuneKnob g_tune_burst_zc{3};              // host bursts: pinned rings read in place by the resident server
thread_local netcsum::TuneKnob g_tune_burst_idle{500};           // resident burst server: idle microseconds before it stops
thread_local netcsum::TuneKnob g_tune_burst_life{1000};          // resident burst server: microseconds of residency per launch
thread_local netcsum::TuneKnob g_tune_pkt_bound{-1};            // run-stream packets: -1 auto, 0..3, 4 ring plans
thread_local netcsum::TuneKnob g_tune_tx_passes{0};             // run-stream Tx: 0 auto (2 passes), 1, 2
std::atomic<int> g_err_reports{0};

NET_ERR dev_fail(const char* what, hipError_t e) {
    if (g_err_reports.fetch_add(1) < 8) {
        std::fprintf(stderr, "[netcsum-mi355x] %s failed: %s (%d) — no CPU fallback, returning "
                             "NET_UTIL_ERR_MI355X_DEV\n", what, hipGetErrorString(e), (int)e);
    }
    return (NET_ERR)NET_UTIL_ERR_MI355X_DEV;
}

#define NC_HIP(call)                                    \
    do {                                                \
        hipError_t e_ = (call);                         \
        if (e_ != hipSuccess) return dev_fail(#call, e_); \
    } while (0)

int cu_count(int dev) {
    static std::atomic<int> cache[kMaxDev];
    if (dev < 0 || dev >= kMaxDev) return 256;
    int v = cache[dev].load();
    if (v <= 0) {
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) {
            v = 256;
        }
        cache[dev].store(v);
    }
    return v;
}

int pow2_group(uint32_t want) {                     // smallest supported group >= want
    static const int gs[] = {1, 4, 8, 16, 32, 64};
    for (int g : gs) {
        if ((uint32_t)g >= want) return g;
    }
    return 64;
}

int chunk_slots(uint32_t want) {                    // smallest supported K >= want
    static const int ks[] = {1, 2, 3, 4, 6, 8};
    for (int k : ks) {
        if ((uint32_t)k >= want) return k;
    }
    return 8;
}

uint32_t gcd_u32(uint32_t a, uint32_t b) {
    while (b) {
        const uint32_t t = a % b;
        a = b;
        b = t;
    }
    return a;
}

// v4 (wave-tile LDS image) geometry for a strided batch, if one compiled instantiation fits:
// G lanes per segment (S = 64/G segments per wave-tile), P KiB image per stage, K chunks per lane.
bool choose_tile(const netcsum::SegBatchArgs& a, int g_force, int k_force, int* g_out, int* p_out, int* k_out) {
    if (a.seg_off != nullptr || a.seg_stride < a.seg_len || a.seg_stride > 0xFFFFFFFFull) return false;
    const uint32_t stride = (uint32_t)a.seg_stride;
    const uint32_t g16 = stride ? gcd_u32(stride, 16u) : 16u;
    const uint32_t maxlead = (uint32_t)((uintptr_t)a.base % g16) + (16u - g16);   // worst first-chunk offset
    const uint32_t nchmax = (maxlead + a.seg_len + 15u) >> 4;
    static const int gs[] = {1, 4, 8, 16, 32, 64};
    static const int ps[] = {1, 2, 4, 6, 8};
    static const int ks[] = {1, 2, 3, 4, 6, 8};
    for (int g : gs) {
        if (g_force && g != g_force) continue;
        const uint32_t S = 64u / (uint32_t)g;
        const uint64_t img = (uint64_t)(S - 1u) * stride + a.seg_len + 127u;
        const uint64_t pimg = a.pseudo ? (uint64_t)(S - 1u) * a.pseudo_stride + a.pseudo_len + 15u : 0u;
        if (pimg > 1024u) continue;
        const uint32_t kneed = (nchmax + (uint32_t)g - 1u) / (uint32_t)g;
        if (!g_force && kneed > 8u) continue;            // prefer the narrowest group that fits
        for (int p : ps) {
            if ((uint64_t)p * 1024u < img) continue;
            for (int k : ks) {
                if (k_force && k != k_force) continue;
                if ((uint32_t)k < kneed) continue;
                if (netcsum::tile_supported(g, p, k)) {
                    *g_out = g;
                    *p_out = p;
                    *k_out = k;
                    return true;
                }
            }
        }
    }
    return false;
}

// Geometry policy (round-1 measurements on MI355X, profiles/r1_sweep_*.jsonl):
//  * kernel 2 (pipelined register loads) is the fastest form for C2, C3 and C4;
//  * G = narrowest lane group whose 8 chunk slots per lane cover a segment (1500 B -> G 16, K 6;
//    20-B headers -> G 1, K 2), from the exact worst-case chunk count of the batch's alignment;
//  * contiguous block tiles of 4 segments per group (grid = n / (groups per block * 4));
//  * non-temporal loads when G >= 8 (lane groups share no 16-B chunks); plain loads for narrow
//    groups, whose neighbouring lanes re-read shared chunks through L1/L2.
netcsum::LaunchCfg choose_cfg(int dev, const netcsum::SegBatchArgs& a, uint32_t len_hint) {
    const bool varlen = a.seg_off != nullptr;
    netcsum::LaunchCfg c{};
    c.block = g_tune_block.load();
    if (c.block < 64 || c.block > 1024 || (c.block & 63)) c.block = 256;
    c.kernel = g_tune_kernel.load();
    c.cus = cu_count(dev);
    c.grid_mult = g_tune_grid_mult.load();
    c.grid = g_tune_grid.load();                       // > 0: fixed grid (grid-stride mode)
    const int tile = g_tune_tile.load();
    c.tile = tile >= 0 ? tile : (c.grid > 0 ? 0 : 4);
    const int nt = g_tune_nt.load();

    if (c.kernel == 0) {
        c.kernel = netcsum::hdrstream_supported(a) ? 8
                 : netcsum::hdr_supported(a) ? 7
                 : netcsum::small_supported(a) ? 5
                 : (netcsum::stream_dense(a) || (varlen && netcsum::stream_supported(a))) ? 6 : 2;
    }
    if (c.kernel == 8) {
        if (netcsum::hdrstream_supported(a)) {
            // Run-stream header form (the default for packed 16 / 20-B headers, C3): TILE > 0 =
            // headers per wave run, CHUNKS 4 / 8 = pieces in flight (auto 4), non-temporal loads
            // unless NT_LOADS 0. Auto run: the most headers (multiple of 16) whose bytes fit the 4
            // pieces in flight from any 128-B lead, so a wave reads its run in ONE round: 192 x 20 B
            // with the row touch = 0.0583 ms against 0.0627 for kernel 7 (r2c3u / r2c3p sweeps).
            int d = g_tune_chunks.load();
            c.chunks_per_pass = (d == 8) ? 8 : 4;
            c.stream_spw = tile > 0 ? (uint32_t)tile : ((4096u - 128u) / a.seg_len) & ~15u;
            c.nt = nt != 0;
            c.group_lanes = 64;
            c.blocks_needed = 0;
            return c;
        }
        c.kernel = 7;                                  // outside its domain: the LDS-tile header form
    }
    if (c.kernel == 7) {
        if (netcsum::hdr_supported(a)) {
            // Defaults from the r2 sweeps (C3, 16 M x 20 B, tools/c3_sweep.py): 4 headers per lane
            // (256-header tiles = 5 whole KiB now that the piece count is exact), 2 tiles in flight,
            // 2 tiles per wave (grid = tiles / 8): 0.0615 ms = 6.0 TB/s vs 0.063 for round 1's 2
            // headers x 3 tiles x 4 tiles per wave; GRID_MULT > 1 instead sizes the grid as resident
            // blocks x CUs x mult.
            const bool auto_h = !(tile == 1 || tile == 2 || tile == 4);
            c.tile = netcsum::hdr_lanes_h(a, auto_h ? 4 : tile);   // TILE = headers per lane (1, 2, 4)
            int st = g_tune_chunks.load();
            if (!(st == 2 || st == 3 || st == 4)) st = (c.tile == 2) ? 3 : 2;
            c.chunks_per_pass = st;
            c.group_lanes = 1;
            c.nt = true;
            c.blocks_needed = 0;
            if (c.grid <= 0) {
                const uint64_t tiles = ((uint64_t)a.n_seg + 64u * c.tile - 1u) / (64u * c.tile);
                const uint64_t per_wave = (auto_h && c.tile == 4) ? 2u : 4u;
                c.grid = c.grid_mult > 1 ? netcsum::hdr_occupancy(a, st, c.tile) * c.cus * c.grid_mult
                                         : (int)std::max<uint64_t>(1u, (tiles + 4u * per_wave - 1u) / (4u * per_wave));
            }
            return c;
        }
        c.kernel = 5;                                  // outside its domain: the register form
    }
    if (c.kernel == 6) {
        if (netcsum::stream_supported(a)) {
            int d = g_tune_chunks.load();
            if (!(d == 4 || d == 6 || d == 8)) d = 4;
            c.chunks_per_pass = d;
            c.nt = nt != 0;                                // default non-temporal: the run is read once
            // Run length (segments per wave): TILE > 0 sets it; GRID_BLOCKS > 0 forces 4 x grid runs;
            // GRID_MULT > 1 sizes runs for that many rounds of resident waves; default 16 segments
            // (r1w5 sweep, C2: runs of 16 read 6.8 TB/s, single-round runs of 128 6.6 TB/s — short
            // runs keep the waves in flight on nearby bytes).
            uint64_t waves;
            if (tile > 0) {
                waves = ((uint64_t)a.n_seg + (uint64_t)tile - 1u) / (uint64_t)tile;
            } else if (c.grid > 0) {
                waves = 4ull * (uint64_t)c.grid;
            } else if (c.grid_mult > 1) {
                waves = (uint64_t)netcsum::stream_occupancy(d, a, c.nt) * 4u * (uint64_t)c.cus * (uint64_t)c.grid_mult;
            } else {
                // runs of 16 segments for dense batches (C2); varlen ones (C4) size their runs on the
                // device to about RUN_BYTES (launch_batch), the grid covering the shortest run, or take
                // runs of 8 (r2ct) with VARLEN_RUN_BYTES 0
                c.run_bytes = varlen ? netcsum::varlen_run_bytes() : 0u;
                uint64_t run = !varlen ? 16u : c.run_bytes ? netcsum::kVarlenSpwMin : 8u;
                if (!varlen) {
                    // a run whose bytes are a multiple of 16 KiB (16 x 1 / 2 / 4 / 8 KiB segments) or
                    // past 48 KiB (9000-B jumbo frames) runs at 79-87 % of spec against 90-91 % for
                    // runs of about 20 KiB that are not (profiles/r6zq_seglen.jsonl: 1024 B x 16
                    // 0.2397 ms, x 20 0.2091; 4096 x 16 0.2183, x 5 0.2069; 9000 x 16 0.2359, x 2
                    // 0.2071); C2's 16 x 1500 B stays
                    const uint64_t st = a.seg_stride ? a.seg_stride : a.seg_len;
                    if ((16u * st) % 16384u == 0u || 16u * st > 49152u) {
                        run = std::max<uint64_t>(1u, (20480u + st / 2u) / st);
                        if ((run * st) % 16384u == 0u && st % 16384u != 0u) run += 1u;
                    }
                }
                if (!varlen) {                         // small batches: latency-bound runs halve until
                    while (run > 1u && (uint64_t)a.n_seg < 2048u * run) run >>= 1;   // >= 2048 waves
                }                                      // (as the packet batches, pkt_batch)
                waves = ((uint64_t)a.n_seg + run - 1u) / run;
            }
            c.stream_spw = netcsum::stream_spw(a, waves);
            c.group_lanes = 64;
            c.blocks_needed = 0;
            return c;
        }
        c.kernel = 2;                                  // varlen, sparse or short segments: general form
    }
    if (c.kernel == 5) {
        if (netcsum::small_supported(a)) {
            c.group_lanes = 1;
            c.chunks_per_pass = (int)((a.seg_len + 3u) >> 2);   // dwords per segment
            c.tile = tile >= 0 ? tile : (c.grid > 0 ? 0 : 1);   // one pass: r1u sweep (C3)
            c.nt = false;
            c.blocks_needed = 0;
            return c;
        }
        c.kernel = 2;                                  // not small / aligned: general form
    }
    if (c.kernel == 4) {
        int g = 0, p = 0, k = 0;
        if (choose_tile(a, g_tune_group.load(), g_tune_chunks.load(), &g, &p, &k)) {
            c.group_lanes = g;
            c.tile_pieces = p;
            c.chunks_per_pass = k;
            c.block = 256;                             // 4 independent waves per block
            c.blocks_needed = 0;
            c.nt = nt != 0;
            return c;
        }
        c.kernel = 2;                                  // varlen, or no instantiation fits
    }
    uint32_t chunks;                                   // worst-case 16-B chunks per segment
    if (varlen) {
        chunks = 288u;                                 // assume the C4 mean (~4.5 KB)
    } else {
        const uint32_t stride = (uint32_t)a.seg_stride;
        const uint32_t g16 = stride ? gcd_u32(stride, 16u) : 16u;
        const uint32_t maxlead = (uint32_t)((uintptr_t)a.base % g16) + (16u - g16);
        chunks = (maxlead + len_hint + 15u) >> 4;
        if (chunks == 0u) chunks = 1u;
    }
    const uint32_t kmax = (c.kernel == 2 || c.kernel == 3) ? 8u : 4u;
    int g = g_tune_group.load();
    if (g == 0) {
        g = varlen ? 32 : pow2_group((chunks + kmax - 1u) / kmax);
    }
    g = pow2_group((uint32_t)g);
    c.group_lanes = g;
    int k = g_tune_chunks.load();
    if (k == 0) {
        k = chunk_slots(std::min<uint32_t>(kmax, std::max<uint32_t>(1u, (chunks + (uint32_t)g - 1u) / (uint32_t)g)));
    }
    c.chunks_per_pass = k;
    c.nt = nt >= 0 ? (nt != 0) : (g >= 8);
    const uint32_t gpb = (uint32_t)(c.block / g);
    c.blocks_needed = ((uint64_t)a.n_seg + gpb - 1u) / gpb;
    return c;
}

NET_ERR check_op(NETCSUM_OP op, const void* d_pseudo, CPU_INT16U pseudo_len) {
    if ((int)op < 0 || (int)op > 3) return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
    if ((op == NETCSUM_OP_HDR_CALC || op == NETCSUM_OP_HDR_VERIFY) && d_pseudo != nullptr && pseudo_len != 0) {
        return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;     // header checksums take no pseudo-header
    }
    return NET_UTIL_ERR_NONE;
}

// Device scratch of the packet batches (two-pass Tx records, the walk pass's flags when the caller
// passes none) and of the varlen run word: plain hipMalloc memory (memory from the stream-ordered
// allocator measured ~70 us slower for the record stores on 1 M packets, profiles/r2tx_*), one buffer
// per (device, stream), kept PER HOST THREAD: only the calling thread hands a buffer out, launches on
// it and evicts it, so no other thread can free it between the hand-out and the launches that use it.
// A lease records an event on the stream after the launches that use its buffer; evicting (least
// recently used, beyond kScratchSlots) or growing a buffer waits for that event — never for the whole
// device — and a new lease whose earlier launches are still pending makes the stream wait for it, so
// a stream created with the handle of a destroyed one whose work is still running cannot overtake it.
// Under stream capture no event is recorded and the slot is pinned (the captured graph keeps its
// address): capture needs one uncaptured call first. Later uncaptured calls on that stream get a slot
// of their own. A graph's replays share its pinned buffer with each other, so replays of one graph
// must be ordered (one stream, or events) — as for any graph that writes a buffer.
constexpr int kScratchSlots = 16;
struct ScratchSlot {
    int                dev = -1;
    hipStream_t        stream = nullptr;
    void*              p = nullptr;
    size_t             cap = 0;
    uint64_t           used = 0;
    hipEvent_t         ev = nullptr;  // recorded after the last launches that used p
    bool               ev_live = false;
    bool               pinned = false;  // used under stream capture: never freed while the thread runs
    bool               unordered = false;  // used by a lease with no event since the last record
    bool               tail_dirty = false; // tail words handed out by a call that did not confirm the
                                           // launch of the pass that resets them (ScratchLease::tail_words)
    uint32_t           seq = 0;         // last tag handed out (ScratchLease::next_tag)
};

hipError_t slot_wait(ScratchSlot& sl) {                // all launches that used sl.p have finished
    hipError_t e = hipSuccess;
    if (sl.unordered) {
        e = hipDeviceSynchronize();                    // (the caller has made sl.dev current)
        sl.unordered = false;
    } else if (sl.ev_live) {
        e = hipEventSynchronize(sl.ev);
    }
    sl.ev_live = false;
    return e;
}

struct ScratchCache {
    ScratchSlot slots[kScratchSlots];
    uint64_t    tick = 0;

    void drop(ScratchSlot& sl) {                       // free a slot's buffer and event (its device)
        int cur = -1;
        const bool have = hipGetDevice(&cur) == hipSuccess;
        if (sl.dev >= 0) (void)hipSetDevice(sl.dev);
        (void)slot_wait(sl);
        if (sl.p) (void)hipFree(sl.p);
        if (sl.ev) (void)hipEventDestroy(sl.ev);
        if (have && cur >= 0 && cur != sl.dev) (void)hipSetDevice(cur);
        sl = ScratchSlot{};
    }
    void release_all() {
        for (ScratchSlot& sl : slots) {
            if (sl.p || sl.ev) drop(sl);
        }
    }
    ~ScratchCache() { release_all(); }
};

thread_local ScratchCache tls_scratch;

// A buffer of >= `bytes` for launches on stream `st` of device `dev`; end() (or the destructor) after
// the last launch that uses it records the slot's event. An UNORDERED lease (ordered = false) is for
// contents any interleaving leaves correct (the varlen run word: any value is a valid run length):
// it records no event (an event record costs ~3 us of GPU time per call, profiles/r3d_event_probe)
// and its slot is freed after a device synchronisation instead.
constexpr size_t kTailBytes = 64;

class ScratchLease {
public:
    hipError_t acquire(int dev, hipStream_t st, size_t bytes, bool ordered = true) {
        stream_ = st;
        ordered_ = ordered;
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (st != nullptr && hipStreamIsCapturing(st, &cs) != hipSuccess) cs = hipStreamCaptureStatusNone;
        capturing_ = cs != hipStreamCaptureStatusNone;
        ScratchCache& c = tls_scratch;
        ScratchSlot* hit = nullptr;
        ScratchSlot* lru = nullptr;
        for (ScratchSlot& sl : c.slots) {
            // a slot pinned by a capture belongs to its graph: a direct (uncaptured) call on the same
            // stream takes a slot of its own, so it can grow it and never shares the graph's buffer
            if (sl.p != nullptr && sl.dev == dev && sl.stream == st && (capturing_ || !sl.pinned)) {
                hit = &sl;
                break;
            }
            if (sl.pinned) continue;
            if (lru == nullptr || sl.p == nullptr || (lru->p != nullptr && sl.used < lru->used)) lru = &sl;
        }
        if (hit == nullptr) {
            if (lru == nullptr) return hipErrorOutOfMemory;           // every slot pinned by captures
            if (lru->p != nullptr || lru->ev != nullptr) c.drop(*lru);  // evict: waits for its event
            hit = lru;
            hit->dev = dev;
            hit->stream = st;
        }
        if (hit->cap < bytes + kTailBytes) {
            if (capturing_ || hit->pinned) return hipErrorStreamCaptureUnsupported;   // no allocation under capture
            hipError_t e = slot_wait(*hit);                // the stream's earlier launches may use it
            if (e != hipSuccess) return e;
            if (hit->p) (void)hipFree(hit->p);
            hit->p = nullptr;
            hit->cap = 0;
            const size_t cap = std::max<size_t>(bytes + kTailBytes, (size_t)1 << 20);
            e = hipMalloc(&hit->p, cap);
            if (e != hipSuccess) {
                hit->p = nullptr;
                return e;
            }
            // the tail words start at zero (tail_words: counters that their users reset themselves)
            e = hipMemsetAsync(static_cast<uint8_t*>(hit->p) + cap - kTailBytes, 0, kTailBytes, st);
            if (e != hipSuccess) {
                (void)hipFree(hit->p);
                hit->p = nullptr;
                return e;
            }
            hit->cap = cap;
            hit->tail_dirty = false;
        }
        if (hit->tail_dirty) {
            // the last call that used the tail words (the offset/length deferral counters) failed
            // between the kernel that counts up and the pass that resets them: zero them in stream
            // order before this call's launches (a stale count re-ran stale list entries)
            hipError_t e = hipMemsetAsync(static_cast<uint8_t*>(hit->p) + hit->cap - kTailBytes, 0, kTailBytes, st);
            if (e != hipSuccess) return e;
            hit->tail_dirty = false;
        }
        if (ordered && hit->ev_live && !capturing_ && hipEventQuery(hit->ev) == hipErrorNotReady) {
            hipError_t e = hipStreamWaitEvent(st, hit->ev, 0);
            if (e != hipSuccess) return e;
        }
        if (hit->ev == nullptr && !capturing_ && ordered) {
            hipError_t e = hipEventCreateWithFlags(&hit->ev, hipEventDisableTiming);
            if (e != hipSuccess) return e;
        }
        hit->used = ++c.tick;
        if (capturing_) hit->pinned = true;
        if (!ordered) hit->unordered = true;
        slot_ = hit;
        return hipSuccess;
    }
    void* ptr() const { return slot_ ? slot_->p : nullptr; }
    // The slot's last kTailBytes, past every request (zeroed when the slot is allocated): words that
    // outlive a call — the offset/length deferral counter, which the deferred pass resets to zero.
    // Handing them out marks the slot dirty until tail_reset_enqueued(): a call that fails before its
    // resetting pass is enqueued leaves them to be zeroed by the next acquire() of the slot.
    uint32_t* tail_words() const {
        if (slot_ == nullptr) return nullptr;
        slot_->tail_dirty = true;
        return reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(slot_->p) + slot_->cap - kTailBytes);
    }
    void tail_reset_enqueued() {
        if (slot_) slot_->tail_dirty = false;
    }
    // A tag no earlier call on this slot used (a deferral word holding it was written by this call;
    // after 2^32 calls a stale word may match once, which only repeats an idempotent pass).
    uint32_t next_tag() {
        if (++slot_->seq == 0u) slot_->seq = 1u;
        return slot_->seq;
    }
    hipError_t end() {
        ScratchSlot* sl = slot_;
        slot_ = nullptr;
        if (sl == nullptr || capturing_ || !ordered_) return hipSuccess;
        const hipError_t e = hipEventRecord(sl->ev, stream_);
        sl->ev_live = e == hipSuccess;
        return e;
    }
    ~ScratchLease() { (void)end(); }

private:
    ScratchSlot* slot_ = nullptr;
    hipStream_t  stream_ = nullptr;
    bool         capturing_ = false;
    bool         ordered_ = true;
};

// (NETCSUM_TUNE_STREAM_WAVES set: measurements of fixed residencies take no plans)
static bool g_tune_stream_waves_set() {
    return netcsum::stream_waves_tuned();
}

// ---- ring plans (netcsum_pktstream.hip pkt_plan_block): the form and run length the last batch on a
// ring sampled for the next one. The words live in one pinned, coherent, device-mapped allocation per
// device that is never freed (a launch still in flight may store into its word after its thread has
// gone); each thread keeps a small table of its rings, each with a word and a tag (a word reused for
// another ring, or a late store of an evicted one, carries another tag and is ignored).
constexpr uint32_t kPlanWords = 4096u;
struct PlanPool {
    std::once_flag once;
    uint32_t* h = nullptr;
    uint32_t* d = nullptr;
};
PlanPool g_plan_pool[kMaxDev];
std::atomic<uint32_t> g_plan_next{0};
struct RingPlan {
    int dev = -1;
    const void* base = nullptr;
    uint64_t stride = 0;
    uint32_t pkt_len = 0, n = 0, slot = 0, tag = 0, plan = 0, use = 0, calls = 0;
    int ip_ver = -1;
    uint32_t plan_id = 0;
};
constexpr int kRingPlans = 16;
thread_local RingPlan tls_ring_plans[kRingPlans];
thread_local uint32_t tls_ring_clock = 0;
// NetUtil_MI355X_PlanBind: the caller's identity for the layout its next batches carry (0: none, the
// plans are keyed on the batch's addresses alone). Part of every plan key, so two layouts placed at the
// same addresses under different ids keep a plan each and never run in the other's form.
thread_local uint32_t tls_plan_id = 0;
// NETCSUM_TUNE_PLAN_AHEAD: -1 auto (a batch whose plan has no word yet samples its layout first, in a
// one-block launch the host waits for, from kPlanAheadRing frames / kPlanAheadPool segments), 0 never
// (the first batch runs unplanned and leaves the plan for the next), 1 always.
thread_local netcsum::TuneKnob g_tune_plan_ahead{-1};
constexpr uint32_t kPlanAheadRing = 1u << 22;
constexpr uint32_t kPlanAheadPool = 1u << 19;

// The plan the ring's previous batch left (0: none yet), its word (host and device addresses) and tag
// for this batch's plan block; *d_word = nullptr when no pool could be had (the batch then runs
// without a plan block).
static uint32_t ring_plan(int dev, const void* base, uint64_t stride, uint32_t pkt_len, uint32_t n, int ip_ver,
                          uint32_t** h_word, uint32_t** d_word, uint32_t* tag, uint32_t* calls = nullptr) {
    *h_word = *d_word = nullptr;
    if (dev < 0 || dev >= kMaxDev) return 0u;
    PlanPool& pool = g_plan_pool[dev];
    std::call_once(pool.once, [&]() {
        void* h = nullptr;
        void* dp = nullptr;
        if (hipHostMalloc(&h, kPlanWords * sizeof(uint32_t), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
            (void)hipGetLastError();
            return;
        }
        if (hipHostGetDevicePointer(&dp, h, 0) != hipSuccess) {
            (void)hipGetLastError();
            return;
        }
        std::memset(h, 0, kPlanWords * sizeof(uint32_t));
        pool.h = static_cast<uint32_t*>(h);
        pool.d = static_cast<uint32_t*>(dp);
    });
    if (pool.h == nullptr) return 0u;
    RingPlan* e = nullptr;
    RingPlan* lru = &tls_ring_plans[0];
    for (RingPlan& r : tls_ring_plans) {
        if (r.dev == dev && r.base == base && r.stride == stride && r.pkt_len == pkt_len && r.n == n && r.ip_ver == ip_ver &&
            r.plan_id == tls_plan_id) {
            e = &r;
            break;
        }
        if (r.use < lru->use) lru = &r;
    }
    if (e == nullptr) {                                     // a new ring: a fresh word and tag
        e = lru;
        const uint32_t k = g_plan_next.fetch_add(1u);
        *e = RingPlan{};
        e->dev = dev;
        e->base = base;
        e->stride = stride;
        e->pkt_len = pkt_len;
        e->n = n;
        e->ip_ver = ip_ver;
        e->plan_id = tls_plan_id;
        e->slot = k % kPlanWords;
        e->tag = (k / kPlanWords * 2654435761u + k) & 0x7FFFu;
    }
    e->use = ++tls_ring_clock;
    if (calls != nullptr) *calls = e->calls++;
    const uint32_t w = *reinterpret_cast<volatile uint32_t*>(pool.h + e->slot);
    if ((w >> 31) != 0u && ((w >> 16) & 0x7FFFu) == e->tag) e->plan = w & 0xFFFFu;
    *h_word = pool.h + e->slot;
    *d_word = pool.d + e->slot;
    *tag = e->tag;
    return e->plan;
}

// Sample a plan ahead of this batch (NETCSUM_TUNE_PLAN_AHEAD): for a plan entry that has never had a
// word (its first batch), of at least `nmin` items, on a stream that is not being captured.
static bool plan_ahead(hipStream_t s, uint32_t n, uint32_t nmin) {
    const int v = g_tune_plan_ahead.load();
    if (v == 0 || (v < 0 && n < nmin)) return false;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (s != nullptr && hipStreamIsCapturing(s, &cs) != hipSuccess) return false;
    return cs == hipStreamCaptureStatusNone;
}

// The plan word a sampler launch stores for `tag` (coherent host memory, system-scope store), polled:
// the plan (bits 0-15), or 0 when none arrived within limit_ms (the batch then runs unplanned).
static uint32_t wait_plan_word(uint32_t* h_word, uint32_t tag, int limit_ms = 2000) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        const uint32_t w = *reinterpret_cast<volatile uint32_t*>(h_word);
        if ((w >> 31) != 0u && ((w >> 16) & 0x7FFFu) == tag) return w & 0xFFFFu;
        const auto el = std::chrono::steady_clock::now() - t0;
        if (el > std::chrono::milliseconds(limit_ms)) return 0u;
        if (el > std::chrono::microseconds(20)) std::this_thread::yield();
    }
}

NET_ERR launch_batch(const netcsum::SegBatchArgs& a0, uint32_t len_hint, hipStream_t s) {
    int dev = 0;
    NC_HIP(hipGetDevice(&dev));
    netcsum::LaunchCfg c = choose_cfg(dev, a0, len_hint);
    netcsum::SegBatchArgs a = a0;
    const int tile_k = g_tune_tile.load();
    const bool fixed = c.run_bytes == 0u && tile_k >= 1 && tile_k <= 64;    // TUNE_TILE: fixed runs, both forms
    if (c.kernel == 6 && a.seg_off != nullptr && (c.run_bytes != 0u || fixed)) {
        // The batch's plan (varlen_runlen_kernel / the live kernel's sampler block, keyed on its
        // descriptor arrays like the packet rings' plans). Segments with gaps between them — one per
        // pool buffer — in address order take the live-sector stream (plan 3: seg_live_varlen_kernel,
        // the plan's run length and depth; TUNE_TILE 1..64 / TUNE_CHUNKS 4 or 8 override them), which
        // samples the descriptors again in one extra block, so the plan follows the descriptors from
        // batch to batch. Pools too sparse for it take the lane-group pipe form (16 lanes x 6 chunks
        // for >= 1 KiB segments, 8 x 8 for shorter ones), every 4th batch the stream form with the
        // sampler again (a plan left by other descriptors at the same addresses lasts at most 3
        // batches; the sampler costs a 1-block launch, ≈ 5 µs).
        uint32_t* h_word = nullptr;
        uint32_t* d_word = nullptr;
        uint32_t tag = 0u, calls = 0u;
        uint32_t plan = ring_plan(dev, a.base, reinterpret_cast<uint64_t>(a.seg_off), 0xFFFFFFFEu, a.n_seg, -2,
                                  &h_word, &d_word, &tag, &calls);
        const char* ahead = "";
        if (plan == 0u && calls == 0u && d_word != nullptr && !fixed && plan_ahead(s, a.n_seg, kPlanAheadPool)) {
            // the first batch on these descriptors: the sampler alone, waited for, so that this batch
            // already runs in its plan (a one-block launch and a poll of the word)
            ScratchLease word;
            NC_HIP(word.acquire(dev, s, 256u, false));
            uint32_t* run = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(word.ptr()) + 128);
            *reinterpret_cast<volatile uint32_t*>(h_word) = 0u;
            NC_HIP(netcsum::launch_varlen_runlen(a.seg_off, a.seg_len_v, a.n_seg, a.pseudo ? a.pseudo_len : 0u, c.run_bytes,
                                                 c.stream_spw, run, d_word, tag, s));
            NC_HIP(word.end());
            plan = wait_plan_word(h_word, tag);
            ahead = " ahead";
            calls = 1u;                                   // (the pipe form below may use its plan at once)
        }
        if ((plan & 3u) == 3u && d_word != nullptr && g_tune_kernel.load() == 0 && g_tune_group.load() == 0) {
            const int ch = g_tune_chunks.load();
            const uint32_t spw = fixed ? (uint32_t)tile_k : std::min<uint32_t>(64u, std::max<uint32_t>(1u, (plan >> 8) & 0xFFu));
            const int depth = (ch == 4 || ch == 8) ? ch : ((plan & 4u) ? 8 : 4);
            a.plan_out = d_word;
            a.plan_tag = tag;
            NC_HIP(netcsum::launch_live_varlen(a, depth, spw, s));
            char d[192];
            snprintf(d, sizeof d, "seg_live_varlen_kernel<D=%d%s,nt> block=256 segs_per_wave=%u plan=pool(live)%s", depth,
                     (a.pseudo && a.pseudo_len) ? ",pseudo" : "", spw, ahead);
            netcsum::set_last_launch(d);
            return NET_UTIL_ERR_NONE;
        }
        if (!fixed && (plan & 3u) != 0u && (plan & 3u) != 3u && (calls & 3u) != 0u && g_tune_kernel.load() == 0 && g_tune_group.load() == 0 &&
            g_tune_chunks.load() == 0) {                 // (any of those tuned: the form asked for)
            const int k0 = g_tune_kernel.load();
            g_tune_kernel.store(2);
            g_tune_group.store((plan & 3u) == 1u ? 16 : 8);   // plan 1: >= 1 KiB segments, 2: shorter
            g_tune_chunks.store((plan & 3u) == 1u ? 6 : 8);
            const netcsum::LaunchCfg cp = choose_cfg(dev, a0, len_hint);
            g_tune_kernel.store(k0);
            g_tune_group.store(0);
            g_tune_chunks.store(0);
            NC_HIP(netcsum::launch_seg_batch(a, cp, s));
            char d[192];
            snprintf(d, sizeof d, "%s plan=pool(pipe)%s", NetUtil_MI355X_LastLaunch(), ahead);
            netcsum::set_last_launch(d);
            return NET_UTIL_ERR_NONE;
        }
        // adaptive varlen runs: a one-block kernel samples the lengths and leaves the run length in
        // this stream's scratch word, which the batch kernel reads (stream order; any value is safe:
        // the kernel never runs shorter runs than its grid covers), and the plan for the next batch
        // (at +128 of the slot's reserved 256-B header: the lane-group walk pass keeps its deferral word
        // at +0; the packet stream's Tx records and deferred-run list start at +256)
        ScratchLease word;
        NC_HIP(word.acquire(dev, s, 256u, false));
        uint32_t* run = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(word.ptr()) + 128);
        NC_HIP(netcsum::launch_varlen_runlen(a.seg_off, a.seg_len_v, a.n_seg, a.pseudo ? a.pseudo_len : 0u, c.run_bytes,
                                             c.stream_spw, run, d_word, tag, s));
        a.run_dev = fixed ? nullptr : run;                 // (fixed runs: the sampler for the plan only)
        NC_HIP(netcsum::launch_seg_batch(a, c, s));
        NC_HIP(word.end());
        return NET_UTIL_ERR_NONE;
    }
    NC_HIP(netcsum::launch_seg_batch(a, c, s));
    return NET_UTIL_ERR_NONE;
}

// ----------------------------------------------------------- per-thread host-path contexts
// One context per (host thread, device): its own stream, pinned staging, completion word and
// device buffers, so one host thread per device needs no lock (SURVEY §8(b) threading). The
// context is released when its thread exits (thread_local destructor) or on request
// (NetUtil_MI355X_ThreadRelease); a partially failed initialisation is rolled back.
struct HostCtx {
    bool                 ready = false;
    int                  dev = -1;
    hipStream_t          stream = nullptr;
    uint8_t*             h_stage = nullptr;   // pinned
    uint8_t*             d_stage = nullptr;
    size_t               cap = 0;
    unsigned long long*  d_sum = nullptr;
    unsigned long long*  h_sum = nullptr;     // pinned, mapped
    unsigned long long*  h_sum_dev = nullptr; // device alias of h_sum
    uint8_t*             h_stage_dev = nullptr;  // device alias of h_stage (zero-copy reads)
    uint32_t             seq = 0;                 // completion tags of the single-block launches
    // pipelined host batch
    hipStream_t          pstream[3] = {nullptr, nullptr, nullptr};
    uint8_t*             d_pipe[3] = {nullptr, nullptr, nullptr};
    size_t               pipe_cap = 0;
    uint8_t*             h_pipe[3] = {nullptr, nullptr, nullptr};   // pinned descriptor staging per slot
    size_t               hpipe_cap = 0;
    // zero-copy bursts (burst_zero_copy): device results, and coherent pinned memory holding the
    // completion word, the results the completion kernel copies out, and the burst's descriptors
    uint8_t*             d_burst = nullptr;
    uint8_t*             h_burst = nullptr;
    uint8_t*             h_burst_dev = nullptr;
    // resident burst server (TUNE_BURST_ZERO_COPY 3): its stream, whether it may be serving, the last
    // burst number posted
    hipStream_t          sstream = nullptr;
    bool                 server_live = false;
    uint64_t             post_seq = 0;

    bool empty() const {
        if (stream || h_stage || d_stage || d_sum || h_sum || d_burst || h_burst || sstream) return false;
        for (int j = 0; j < 3; ++j) {
            if (pstream[j] || d_pipe[j] || h_pipe[j]) return false;
        }
        return true;
    }
    // Frees everything this context holds (on its own device), leaving it reusable.
    void release() {
        if (empty()) {
            ready = false;
            return;
        }
        int cur = -1;
        const bool have_cur = hipGetDevice(&cur) == hipSuccess;
        if (dev >= 0) (void)hipSetDevice(dev);
        if (stream) (void)hipStreamSynchronize(stream);
        for (int j = 0; j < 3; ++j) {
            if (pstream[j]) (void)hipStreamSynchronize(pstream[j]);
        }
        (void)stop_server(0);                     // (no limit: the server reads h_burst, freed below)
        if (sstream) (void)hipStreamDestroy(sstream);
        if (stream) (void)hipStreamDestroy(stream);
        if (h_stage) (void)hipHostFree(h_stage);
        if (d_stage) (void)hipFree(d_stage);
        if (d_sum) (void)hipFree(d_sum);
        if (h_sum) (void)hipHostFree(h_sum);
        if (d_burst) (void)hipFree(d_burst);
        if (h_burst) (void)hipHostFree(h_burst);
        for (int j = 0; j < 3; ++j) {
            if (pstream[j]) (void)hipStreamDestroy(pstream[j]);
            if (d_pipe[j]) (void)hipFree(d_pipe[j]);
            if (h_pipe[j]) (void)hipHostFree(h_pipe[j]);
        }
        if (have_cur && cur != dev && cur >= 0) (void)hipSetDevice(cur);
        *this = HostCtx{};
    }
    ~HostCtx() { release(); }
    bool stop_server(int limit_ms);
};

thread_local HostCtx tls_ctx[kMaxDev];

NET_ERR host_ctx(HostCtx** out) {
    int dev = 0;
    NC_HIP(hipGetDevice(&dev));
    if (dev < 0 || dev >= kMaxDev) return dev_fail("device index", hipErrorInvalidDevice);
    HostCtx& c = tls_ctx[dev];
    if (!c.ready) {
        c.release();                               // roll back a previous partial initialisation
        c.dev = dev;
        hipError_t e = hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipMalloc(&c.d_sum, 16);
        // coherent: the single-block kernel's system-scope completion store is visible while it runs
        if (e == hipSuccess) e = hipHostMalloc(&c.h_sum, 16, hipHostMallocMapped | hipHostMallocCoherent);
        if (e == hipSuccess) e = hipHostGetDevicePointer(reinterpret_cast<void**>(&c.h_sum_dev), c.h_sum, 0);
        if (e != hipSuccess) {
            c.release();
            return dev_fail("host context init", e);
        }
        c.ready = true;
    }
    *out = &c;
    return NET_UTIL_ERR_NONE;
}

NET_ERR ensure_stage(HostCtx& c, size_t bytes) {
    if (bytes <= c.cap) return NET_UTIL_ERR_NONE;
    size_t cap = std::max<size_t>(bytes, 64u * 1024u);
    cap = (cap + 4095u) & ~(size_t)4095u;
    if (c.h_stage) { (void)hipHostFree(c.h_stage); c.h_stage = nullptr; }
    if (c.d_stage) { (void)hipFree(c.d_stage); c.d_stage = nullptr; }
    c.cap = 0;
    NC_HIP(hipHostMalloc(&c.h_stage, cap, hipHostMallocMapped));
    NC_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&c.h_stage_dev), c.h_stage, 0));
    NC_HIP(hipMalloc(&c.d_stage, cap));
    c.cap = cap;
    return NET_UTIL_ERR_NONE;
}

// The three pipeline slots of a host-memory batch: streams, device buffers of >= dev_bytes and pinned
// descriptor staging of >= host_bytes (grown on demand; the previous call has drained them).
NET_ERR ensure_pipe(HostCtx& c, size_t dev_bytes, size_t host_bytes) {
    for (int j = 0; j < 3; ++j) {
        if (!c.pstream[j]) NC_HIP(hipStreamCreateWithFlags(&c.pstream[j], hipStreamNonBlocking));
    }
    if (dev_bytes > c.pipe_cap) {
        for (int j = 0; j < 3; ++j) {
            if (c.d_pipe[j]) { (void)hipFree(c.d_pipe[j]); c.d_pipe[j] = nullptr; }
        }
        c.pipe_cap = 0;
        for (int j = 0; j < 3; ++j) NC_HIP(hipMalloc(&c.d_pipe[j], dev_bytes));
        c.pipe_cap = dev_bytes;
    }
    if (host_bytes > c.hpipe_cap) {
        for (int j = 0; j < 3; ++j) {
            if (c.h_pipe[j]) { (void)hipHostFree(c.h_pipe[j]); c.h_pipe[j] = nullptr; }
        }
        c.hpipe_cap = 0;
        for (int j = 0; j < 3; ++j) NC_HIP(hipHostMalloc(&c.h_pipe[j], host_bytes, 0));
        c.hpipe_cap = host_bytes;
    }
    return NET_UTIL_ERR_NONE;
}

size_t al256(size_t x) { return (x + 255u) & ~(size_t)255u; }

// A host-memory batch that returns early (any error) first waits for its three pipeline streams, so
// no copy into the caller's memory is still in flight when the call returns. (A Tx batch that fails
// may leave the caller's buffer with some chunks finalized and others not.)
struct PipeDrainOnExit {
    HostCtx& c;
    bool     done = false;
    ~PipeDrainOnExit() {
        if (done) return;
        for (int j = 0; j < 3; ++j) {
            if (c.pstream[j]) (void)hipStreamSynchronize(c.pstream[j]);
        }
    }
};

// One chunk of a host-memory batch: items [s0, s0 + ns) whose bytes are [lo, hi) of the caller's buffer.
struct HostChunk {
    uint32_t s0, ns;
    uint64_t lo, hi;
};

// Chunks of about n / n_chunks items each; items of a strided batch (h_off == NULL) are
// [i * stride, i * stride + len), of an offset/length batch [h_off[i], h_off[i] + h_len[i]).
// Returns the largest chunk's byte span.
uint64_t plan_chunks(const uint64_t* h_off, const uint16_t* h_len, uint64_t stride, uint32_t len, uint32_t n,
                     uint32_t n_chunks, std::vector<HostChunk>& out) {
    if (n_chunks == 0) n_chunks = 1;
    if (n_chunks > n) n_chunks = n;
    const uint32_t per = (n + n_chunks - 1u) / n_chunks;
    uint64_t maxb = 0;
    out.clear();
    for (uint32_t s0 = 0; s0 < n; s0 += per) {
        HostChunk k{s0, std::min(per, n - s0), 0, 0};
        if (h_off == nullptr) {
            k.lo = (uint64_t)s0 * stride;
            k.hi = (uint64_t)(s0 + k.ns - 1u) * stride + len;
        } else {
            k.lo = ~0ull;
            for (uint32_t i = s0; i < s0 + k.ns; ++i) {
                k.lo = std::min<uint64_t>(k.lo, h_off[i]);
                k.hi = std::max<uint64_t>(k.hi, h_off[i] + h_len[i]);
            }
            if (k.hi < k.lo) k.hi = k.lo;
        }
        maxb = std::max<uint64_t>(maxb, k.hi - k.lo);
        out.push_back(k);
    }
    return maxb;
}

}  // namespace

extern "C" {

NET_ERR NetUtil_MI355X_ChkSumBatchStrided(const void* d_seg, uint64_t seg_stride, CPU_INT16U seg_len,
                                          const void* d_pseudo, uint32_t pseudo_stride, CPU_INT16U pseudo_len,
                                          uint32_t n_seg, void* d_out, NETCSUM_OP op, void* hip_stream) {
    NET_ERR e = check_op(op, d_pseudo, pseudo_len);
    if (e != NET_UTIL_ERR_NONE) return e;
    if (n_seg == 0) return NET_UTIL_ERR_NONE;
    if (n_seg > 0x7FFFFFFFu) return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
    if (d_out == nullptr || (d_seg == nullptr && seg_len != 0)) return NET_ERR_FAULT_NULL_PTR;
    netcsum::SegBatchArgs a{};
    a.base = static_cast<const uint8_t*>(d_seg);
    a.seg_stride = seg_stride;
    a.seg_len = seg_len;
    a.pseudo = (pseudo_len != 0) ? static_cast<const uint8_t*>(d_pseudo) : nullptr;
    a.pseudo_stride = pseudo_stride;
    a.pseudo_len = pseudo_len;
    a.n_seg = n_seg;
    a.verify = (op == NETCSUM_OP_DATA_VERIFY || op == NETCSUM_OP_HDR_VERIFY) ? 1u : 0u;
    a.out = d_out;
    return launch_batch(a, seg_len, static_cast<hipStream_t>(hip_stream));
}

NET_ERR NetUtil_MI355X_ChkSumBatchVarLen(const void* d_base, const uint64_t* d_seg_off, const uint16_t* d_seg_len,
                                         const void* d_pseudo, uint32_t pseudo_stride, CPU_INT16U pseudo_len,
                                         uint32_t n_seg, void* d_out, NETCSUM_OP op, void* hip_stream) {
    NET_ERR e = check_op(op, d_pseudo, pseudo_len);
    if (e != NET_UTIL_ERR_NONE) return e;
    if (n_seg == 0) return NET_UTIL_ERR_NONE;
    if (n_seg > 0x7FFFFFFFu) return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
    if (d_out == nullptr || d_base == nullptr || d_seg_off == nullptr || d_seg_len == nullptr) {
        return NET_ERR_FAULT_NULL_PTR;
    }
    netcsum::SegBatchArgs a{};
    a.base = static_cast<const uint8_t*>(d_base);
    a.seg_off = d_seg_off;
    a.seg_len_v = d_seg_len;
    a.pseudo = (pseudo_len != 0) ? static_cast<const uint8_t*>(d_pseudo) : nullptr;
    a.pseudo_stride = pseudo_stride;
    a.pseudo_len = pseudo_len;
    a.n_seg = n_seg;
    a.verify = (op == NETCSUM_OP_DATA_VERIFY || op == NETCSUM_OP_HDR_VERIFY) ? 1u : 0u;
    a.out = d_out;
    return launch_batch(a, 0u, static_cast<hipStream_t>(hip_stream));
}

NET_ERR NetUtil_MI355X_ChkSumBatchStridedHost(const void* h_seg, uint64_t seg_stride, CPU_INT16U seg_len,
                                              const void* h_pseudo, uint32_t pseudo_stride, CPU_INT16U pseudo_len,
                                              uint32_t n_seg, void* h_out, NETCSUM_OP op, uint32_t n_chunks) {
    NET_ERR e = check_op(op, h_pseudo, pseudo_len);
    if (e != NET_UTIL_ERR_NONE) return e;
    if (n_seg == 0) return NET_UTIL_ERR_NONE;
    if (h_out == nullptr || (h_seg == nullptr && seg_len != 0)) return NET_ERR_FAULT_NULL_PTR;
    HostCtx* cp = nullptr;
    e = host_ctx(&cp);
    if (e != NET_UTIL_ERR_NONE) return e;
    HostCtx& c = *cp;
    const bool verify = (op == NETCSUM_OP_DATA_VERIFY || op == NETCSUM_OP_HDR_VERIFY);
    const size_t out_elt = verify ? 1u : 2u;
    const bool has_ph = (h_pseudo != nullptr && pseudo_len != 0);
    if (n_chunks == 0) n_chunks = 1;
    if (n_chunks > n_seg) n_chunks = n_seg;
    const uint32_t per = (n_seg + n_chunks - 1u) / n_chunks;

    // Device layout per in-flight chunk: [segment bytes | pseudo bytes | outputs], 256-B aligned.
    auto al = [](size_t x) { return (x + 255u) & ~(size_t)255u; };
    const size_t seg_bytes = (size_t)(per - 1u) * seg_stride + seg_len;
    const size_t ph_bytes = has_ph ? (size_t)(per - 1u) * pseudo_stride + pseudo_len : 0u;
    const size_t need = al(seg_bytes) + al(ph_bytes) + al((size_t)per * out_elt);
    if (need > c.pipe_cap) {
        for (int j = 0; j < 3; ++j) {
            if (c.d_pipe[j]) { (void)hipFree(c.d_pipe[j]); c.d_pipe[j] = nullptr; }
        }
        c.pipe_cap = 0;
        for (int j = 0; j < 3; ++j) {
            if (!c.pstream[j]) NC_HIP(hipStreamCreateWithFlags(&c.pstream[j], hipStreamNonBlocking));
            NC_HIP(hipMalloc(&c.d_pipe[j], need));
        }
        c.pipe_cap = need;
    }
    int dev = 0;
    NC_HIP(hipGetDevice(&dev));
    for (uint32_t k = 0; k < n_chunks; ++k) {
        const uint32_t s0 = k * per;
        if (s0 >= n_seg) break;
        const uint32_t ns = std::min(per, n_seg - s0);
        const int j = (int)(k % 3u);
        hipStream_t st = c.pstream[j];
        uint8_t* d_seg = c.d_pipe[j];
        uint8_t* d_ph = d_seg + al(seg_bytes);
        uint8_t* d_out = d_ph + al(ph_bytes);
        const size_t sb = (size_t)(ns - 1u) * seg_stride + seg_len;
        NC_HIP(hipMemcpyAsync(d_seg, static_cast<const uint8_t*>(h_seg) + (size_t)s0 * seg_stride, sb,
                              hipMemcpyHostToDevice, st));
        if (has_ph) {
            const size_t pb = (size_t)(ns - 1u) * pseudo_stride + pseudo_len;
            NC_HIP(hipMemcpyAsync(d_ph, static_cast<const uint8_t*>(h_pseudo) + (size_t)s0 * pseudo_stride, pb,
                                  hipMemcpyHostToDevice, st));
        }
        netcsum::SegBatchArgs a{};
        a.base = d_seg;
        a.seg_stride = seg_stride;
        a.seg_len = seg_len;
        a.pseudo = has_ph ? d_ph : nullptr;
        a.pseudo_stride = pseudo_stride;
        a.pseudo_len = has_ph ? pseudo_len : 0u;
        a.n_seg = ns;
        a.verify = verify ? 1u : 0u;
        a.out = d_out;
        // Parity of each segment's start is derived in-kernel from the DEVICE address it reads,
        // so re-basing the chunk at a 256-B aligned device buffer is transparent.
        const netcsum::LaunchCfg cfg = choose_cfg(dev, a, seg_len);
        NC_HIP(netcsum::launch_seg_batch(a, cfg, st));
        NC_HIP(hipMemcpyAsync(static_cast<uint8_t*>(h_out) + (size_t)s0 * out_elt, d_out, (size_t)ns * out_elt,
                              hipMemcpyDeviceToHost, st));
    }
    for (int j = 0; j < 3; ++j) {
        NC_HIP(hipStreamSynchronize(c.pstream[j]));
    }
    return NET_UTIL_ERR_NONE;
}

NET_ERR NetUtil_MI355X_ThreadRelease(void) {
    for (int d = 0; d < kMaxDev; ++d) {
        tls_ctx[d].release();
    }
    tls_scratch.release_all();
    return NET_UTIL_ERR_NONE;
}

NET_ERR NetUtil_MI355X_StreamSum32(const NETCSUM_SPAN* spans, uint32_t n_spans, uint32_t* p_sum32) {
    if (p_sum32 == nullptr || (spans == nullptr && n_spans != 0)) return NET_ERR_FAULT_NULL_PTR;
    HostCtx* cp = nullptr;
    NET_ERR e = host_ctx(&cp);                 // the device must exist even for an empty stream
    if (e != NET_UTIL_ERR_NONE) return e;
    HostCtx& c = *cp;
    size_t total = 0;
    for (uint32_t i = 0; i < n_spans; ++i) total += spans[i].len;
    *p_sum32 = 0u;
    if (total == 0) return NET_UTIL_ERR_NONE;
    const size_t padded = (total + 15u) & ~(size_t)15u;
    if (padded / 16u > 0xFFFFFFFFu) return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
    e = ensure_stage(c, padded);
    if (e != NET_UTIL_ERR_NONE) return e;
    size_t pos = 0;
    for (uint32_t i = 0; i < n_spans; ++i) {
        if (spans[i].len) {
            std::memcpy(c.h_stage + pos, spans[i].p, spans[i].len);
            pos += spans[i].len;
        }
    }
    std::memset(c.h_stage + pos, 0, padded - pos);
    const uint32_t n16 = (uint32_t)(padded / 16u);
    if (padded <= kZeroCopyMax) {
        // one packet (the drop-in's common case): the kernel reads the pinned staging buffer over
        // the bus and stores its single-block total into pinned memory — one launch, one sync
        // the host polls the kernel's tagged completion word instead of synchronising the stream
        // (C1 latency); after 2 s without it, it falls back to the stream sync and its error check
        if (++c.seq == 0u) c.seq = 1u;
        const uint32_t tag = c.seq;
        volatile unsigned long long* w = c.h_sum;
        *w = 0ull;                             // no stale word (e.g. a multi-block sum) can carry the tag
        NC_HIP(netcsum::launch_stream_exact(c.h_stage_dev, n16, c.h_sum_dev, 1, c.stream, tag));
        const auto t0 = std::chrono::steady_clock::now();
        unsigned long long v = *w;
        for (uint32_t spin = 0; (uint32_t)(v >> 32) != tag; ++spin) {
            if ((spin & 1023u) == 1023u && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
                NC_HIP(hipStreamSynchronize(c.stream));
                v = *w;
                if ((uint32_t)(v >> 32) != tag) return dev_fail("completion word", hipErrorUnknown);
                break;
            }
            v = *w;
        }
        *p_sum32 = (uint32_t)v;
        return NET_UTIL_ERR_NONE;
    } else {
        const int grid = (int)std::min<uint32_t>(256u, (n16 + 1023u) / 1024u);
        NC_HIP(hipMemcpyAsync(c.d_stage, c.h_stage, padded, hipMemcpyHostToDevice, c.stream));
        NC_HIP(hipMemsetAsync(c.d_sum, 0, sizeof(unsigned long long), c.stream));
        NC_HIP(netcsum::launch_stream_exact(c.d_stage, n16, c.d_sum, std::max(grid, 2), c.stream));
        NC_HIP(hipMemcpyAsync(c.h_sum, c.d_sum, sizeof(unsigned long long), hipMemcpyDeviceToHost, c.stream));
        NC_HIP(hipStreamSynchronize(c.stream));
    }
    *p_sum32 = (uint32_t)(*(volatile unsigned long long*)c.h_sum);           // the reference's u32 accumulator wraps mod 2^32
    return NET_UTIL_ERR_NONE;
}

NET_ERR NetUtil_MI355X_CRC32BatchStrided(const void* d_base, uint64_t stride, uint32_t len, uint32_t n,
                                         uint32_t* d_out, int cpl, void* hip_stream) {
    if (n == 0) return NET_UTIL_ERR_NONE;
    if (d_out == nullptr || (d_base == nullptr && len != 0)) return NET_ERR_FAULT_NULL_PTR;
    netcsum::CrcBatchArgs a{};
    a.base = static_cast<const uint8_t*>(d_base);
    a.stride = stride;
    a.len = len;
    a.n = n;
    a.cpl = cpl ? 1u : 0u;
    a.out = d_out;
    netcsum::set_last_launch(netcsum::crc_launch_name(len, false));
    int dev = 0;
    NC_HIP(hipGetDevice(&dev));
    NC_HIP(netcsum::launch_crc_batch(a, len, cu_count(dev), static_cast<hipStream_t>(hip_stream)));
    return NET_UTIL_ERR_NONE;
}

NET_ERR NetUtil_MI355X_CRC32BatchVarLen(const void* d_base, const uint64_t* d_off, const uint32_t* d_len, uint32_t n,
                                        uint32_t* d_out, int cpl, void* hip_stream) {
    if (n == 0) return NET_UTIL_ERR_NONE;
    if (d_out == nullptr || d_base == nullptr || d_off == nullptr || d_len == nullptr) return NET_ERR_FAULT_NULL_PTR;
    netcsum::CrcBatchArgs a{};
    a.base = static_cast<const uint8_t*>(d_base);
    a.off = d_off;
    a.lens = d_len;
    a.n = n;
    a.cpl = cpl ? 1u : 0u;
    a.out = d_out;
    netcsum::set_last_launch(netcsum::crc_launch_name(0xFFFFFFFFu, true));
    int dev = 0;
    NC_HIP(hipGetDevice(&dev));
    NC_HIP(netcsum::launch_crc_batch(a, 0xFFFFFFFFu, cu_count(dev), static_cast<hipStream_t>(hip_stream)));
    return NET_UTIL_ERR_NONE;
}

// One CRC-32 (the NetUtil_32BitCRC_Calc register value) of a host buffer: staged into this thread's
// pinned buffer, read from there by the kernel (zero-copy), result copied back.
NET_ERR NetUtil_MI355X_CRC32Host(const void* h_data, uint32_t len, uint32_t* p_crc) {
    if (p_crc == nullptr || (h_data == nullptr && len != 0)) return NET_ERR_FAULT_NULL_PTR;
    HostCtx* cp = nullptr;
    NET_ERR e = host_ctx(&cp);
    if (e != NET_UTIL_ERR_NONE) return e;
    HostCtx& c = *cp;
    *p_crc = 0u;
    if (len == 0) return NET_UTIL_ERR_NONE;
    e = ensure_stage(c, len);
    if (e != NET_UTIL_ERR_NONE) return e;
    std::memcpy(c.h_stage, h_data, len);
    netcsum::CrcBatchArgs a{};
    a.base = c.h_stage_dev;
    a.len = len;
    a.n = 1;
    a.out = reinterpret_cast<uint32_t*>(c.d_sum);
    NC_HIP(netcsum::launch_crc_batch(a, len, cu_count(c.dev), c.stream));
    NC_HIP(hipMemcpyAsync(c.h_sum, c.d_sum, sizeof(uint32_t), hipMemcpyDeviceToHost, c.stream));
    NC_HIP(hipStreamSynchronize(c.stream));
    *p_crc = *reinterpret_cast<volatile uint32_t*>(c.h_sum);
    return NET_UTIL_ERR_NONE;
}

// udp_mode: PktBatchArgs::udp_tx_csum (Tx); d_action / rx_cfg: the Rx burst actions (Rx, optional);
// d_fieldpos: Tx, which fields each packet had written (the host-memory forms' records, optional).
static NET_ERR pkt_batch(const void* d_base, const uint64_t* d_off, const uint16_t* d_len, uint64_t stride,
                         CPU_INT16U pkt_len, uint32_t n_pkt, uint8_t* d_flags, uint32_t udp_mode, bool tx,
                         int ip_ver, void* hip_stream, uint8_t* d_action = nullptr, uint32_t rx_cfg = 0u,
                         uint32_t* d_fieldpos = nullptr, netcsum::PktTxRecord* rec_only = nullptr,
                         int bound_pref = -1) {
    if (n_pkt == 0) return NET_UTIL_ERR_NONE;
    if (n_pkt > 0x7FFFFFFFu) return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
    if (d_base == nullptr || (d_off != nullptr) != (d_len != nullptr) || (!tx && d_flags == nullptr && d_action == nullptr)) {
        return NET_ERR_FAULT_NULL_PTR;
    }
    int dev = 0;
    NC_HIP(hipGetDevice(&dev));
    netcsum::PktBatchArgs a{};
    a.base = static_cast<const uint8_t*>(d_base);
    a.off = d_off;
    a.len = d_len;
    a.stride = stride;
    a.len_u = pkt_len;
    a.n = n_pkt;
    a.flags_out = d_flags;
    a.udp_tx_csum = udp_mode;
    a.action_out = tx ? nullptr : d_action;
    a.rx_cfg = rx_cfg;
    a.fieldpos_out = tx ? d_fieldpos : nullptr;
    netcsum::LaunchCfg c{};
    const uint32_t chunks = d_off ? 288u : ((uint32_t)pkt_len + 30u) / 16u;
    int g = g_tune_group.load();
    if (g < 8) {
        g = d_off ? 32 : std::max(8, pow2_group((chunks + 5u) / 6u));
    }
    c.group_lanes = pow2_group((uint32_t)g);
    c.chunks_per_pass = (int)std::min<uint32_t>(8u, std::max<uint32_t>(1u, (chunks + c.group_lanes - 1u) / c.group_lanes));
    // Strided batches store through a buffer resource based at each wave's first packet of a stage,
    // reaching the stage's other 64/G - 1 packets by 32-bit offsets (netcsum_packets.hip pkt_store):
    // a stride that would wrap them is refused, never silently mis-addressed.
    if (d_off == nullptr && (uint64_t)(64u / (uint32_t)c.group_lanes - 1u) * stride + 65536u >= 0xFFFFFFFFull) {
        return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
    }
    // Rx streams with nt loads; Tx re-writes header lines it has just read and is faster with plain
    // loads (profiles/r1tc_tx_sweep.jsonl: 0.323 vs 0.356 ms at tile 2).
    const int nt = g_tune_nt.load();
    c.nt = nt >= 0 ? (nt != 0) : !tx;
    c.grid = g_tune_grid.load();
    const int tile = g_tune_tile.load();
    // Run-stream form (netcsum_pktstream.hip) for dense strided IPv4 batches unless the lane-group
    // kernel is forced (TUNE_KERNEL 2); TILE > 0 sets its packets per wave run (default 16).
    const int kern = g_tune_kernel.load();
    // Defaults from the r2tx sweep (tools/pkt_stream_probe.py, 1 M x 1500-B IPv4/TCP): runs of 8
    // packets, 4 pieces in flight, nt loads (Rx 0.215 ms); Tx in two passes (checksum pass writing
    // 8-B records + scatter pass: 0.288 ms against 0.296 for in-pass field writes). Mixed rings run
    // both parses in a wave whose lanes disagree on the version, and a run of 16 spreads that over
    // twice the bytes (profiles/r2zb_pkt_stream_mixed_v6_v4.jsonl, alternating ring: Rx 0.243 ->
    // 0.2185 ms, Tx 0.302 -> 0.292); IPv4 and IPv6 alone stay at 8 (16: +0.9 % / +0.2 %). Shorter
    // datagrams need longer runs (a run's cost is per datagram event AND per wave): about 20 KB per
    // run in multiples of 8 datagrams, 8..64 (40 KB in multiples of 16 for mixed rings); r2zq sweep
    // (tools/pkt_run_probe.py): Rx of 256-B datagrams 0.891 -> 0.567 ms, 576-B 0.424 -> 0.29,
    // 1000-B 0.259 -> 0.222; 1500-B keeps 8.
    // IPv6 / mixed batches through the lane-group kernel: a second pass walks the extension-header
    // chains the batch kernel left as EXT_HDR (netcsum_v6walk.hip). It reads the flags, so a Tx batch
    // without d_flags gets them in the stream's scratch buffer. (The run-stream path below walks them
    // inside its own launches.)
    // (an Rx burst without d_flags keeps them there too, or nowhere for IPv4, whose kernels write
    // each action directly)
    const bool walk = ip_ver != 4;
    const bool own_flags = walk && d_flags == nullptr;
    hipStream_t hs = static_cast<hipStream_t>(hip_stream);
    // Which bytes of each slot are read (NETCSUM_TUNE_PKT_BOUND, netcsum_pktstream.hip): by default the
    // whole span for packed batches (0), else the live pieces with piece 0 loaded during the parse (2;
    // since the one-mask sentinel pop it beats form 3 on every ring layout, profiles/r4m_ring_probe.jsonl:
    // 1520-B slots at +14, 1500-B datagrams 0.2177 against 0.2197 ms, the mixed ring 0.1532 against
    // 0.1583, 2-KiB slots at +64 0.2522 against 0.2677); a burst read in place from host memory may
    // prefer the whole-span form 0 (bound_pref: one PCIe round trip). Live-piece runs span at most
    // 63 KiB (kLiveReach).
    const int d = g_tune_chunks.load() == 8 ? 8 : 4;
    // (a packed batch, stride == pkt_len, says every byte is datagram: nothing to skip, form 0;
    // r4f ring probe: 1 M x 1500 B Rx 0.2145 ms against 0.2188 in form 3)
    const bool dense = d_off == nullptr && stride <= (uint64_t)pkt_len + 64u;
    const bool packed = d_off == nullptr && stride == (uint64_t)pkt_len;
    const int tb0 = g_tune_pkt_bound.load();
    const bool bound_default = tb0 < 0 || tb0 == 4;         // (4: ring plans, else as the default)
    int bound = !bound_default ? tb0 : (packed ? 0 : 2);
    if (bound_pref >= 0 && bound_default) {                 // the caller's preference, where it applies
        if (netcsum::pkt_stream_supported(a, ip_ver, bound_pref)) bound = bound_pref;
    }
    if (d == 8 && bound == 1) bound = 2;                    // (8 pieces in flight: forms 0, 2, 3)
    if (!netcsum::pkt_stream_supported(a, ip_ver, bound) && bound >= 1 && dense && bound_default) {
        bound = 0;                                          // datagrams > 64384 B: past the bitmap's reach
    }
    if (kern != 2 && netcsum::pkt_stream_supported(a, ip_ver, bound)) {
        // offset/length runs: 16 datagrams (their lengths are on the device; the device checks each
        // run's order and reach, and takes a run datagram by datagram otherwise)
        // the live-piece forms parse first, so their runs are longer: about 24 KB of strided span, which
        // gives 1520-B slots runs of 16 (the mixed 40/576/1500-B ring: 0.1532 ms against 0.1921 for 8)
        // and 2-KiB slots runs of 8 (0.2522 against 0.2627 for 16; profiles/r4m_ring_probe.jsonl);
        // offset/length runs 16 (32: 64 KiB of 2-KiB slots, past the reach)
        const uint64_t per = d_off ? 2048u : std::max<uint64_t>(a.stride, 1u);
        const uint64_t budget = bound == 0 ? 20480u : d_off ? 32768u : 24576u;
        uint32_t run = ip_ver == 0 ? (uint32_t)std::min<uint64_t>(64u, std::max<uint64_t>(16u, (40960u / per) & ~15ull))
                                   : (uint32_t)std::min<uint64_t>(64u, std::max<uint64_t>(8u, (budget / per) & ~7ull));
        // dense IPv4 / IPv6 runs of long datagrams: a run of 8 whose bytes are a multiple of 16 KiB or
        // past 48 KiB (2 / 4 / 8 KiB, 9000-B datagrams) runs at 78-88 % of spec, runs of about 10 KiB at
        // 88-92 % (profiles/r6zu_pktlen.jsonl: 2048 B x 8 0.2120 ms, x 5 0.2046; 4096 x 8 0.2219, x 2
        // 0.2050; 8192 x 8 0.2393, x 1 0.2042; 9000 x 8 0.2166, x 1 0.2138); 1500 B keeps its 8
        if (ip_ver != 0 && bound == 0 && !d_off && ((uint64_t)run * per % 16384u == 0u || (uint64_t)run * per > 49152u)) {
            run = (uint32_t)std::max<uint64_t>(1u, 10240u / per);
        }
        // small batches (NIC bursts) are latency-bound: a run costs ~run x len / 4 KiB memory round
        // trips, so runs halve until the batch spreads over >= 2048 waves (burst of 256 mixed frames:
        // Rx 19.9 -> 13.3 us, Tx 22.8 -> 15.7 us; 16 Ki frames: runs of 8, 19.2 -> 17.2 us;
        // profiles/r3t_burst_run_probe.jsonl); batches of >= 2048 runs keep the run length above
        uint32_t spw = (tile > 0 && tile <= 64) ? (uint32_t)tile : run;
        if (!(tile > 0 && tile <= 64)) {
            while (spw > 1u && (uint64_t)n_pkt < 2048ull * spw) spw >>= 1;
        }
        // The ring's plan (netcsum_pktstream.hip pkt_plan_block): for strided batches that are not
        // packed — by default from 16 Ki datagrams (smaller ones are bursts, latency-bound, with the
        // runs halved above), always with TUNE_PKT_BOUND 4 — the launch samples its datagrams in one
        // extra block and leaves the form and run length for the next batch on the same ring (same
        // base, stride, bytes present, count, IP version) in coherent host memory; a batch whose ring
        // has a plan runs in it, the first one in the host's default above.
        // Offset/length batches take ring plans too, keyed on their descriptor arrays: the run length
        // (by the streamed bytes, capped by the sampled pitch to the reach) and the residency.
        const bool plan_ring = !packed && bound_pref < 0 && d == 4 && !(tile > 0 && tile <= 64) &&
                               (tb0 == 4 || (tb0 < 0 && n_pkt >= 16384u)) && rec_only == nullptr &&
                               g_tune_stream_waves_set() == false && netcsum::pkt_stream_supported(a, ip_ver, 2);
        const char* plan_note = "";
        const char* ahead_note = "";
        bool vl_wide = true;                             // the deferred pass's grid: wide unless the plan
        bool vl_inline = false;                          // found the ring's descriptors in order; a dense
        if (plan_ring) {                                 // ring in order: the inline form (pkt_stream_kernel DEF)
            uint32_t run0 = 0u;
            if (d_off == nullptr && netcsum::pkt_stream_supported(a, ip_ver, 0)) {
                run0 = ip_ver == 0 ? (uint32_t)std::min<uint64_t>(64u, std::max<uint64_t>(16u, (40960u / per) & ~15ull))
                                   : (uint32_t)std::min<uint64_t>(64u, std::max<uint64_t>(8u, (20480u / per) & ~7ull));
                while (run0 > 1u && (uint64_t)n_pkt < 2048ull * run0) run0 >>= 1;
            }
            uint64_t cap = d_off ? 64u : (netcsum::kLiveReach - 128u - (uint64_t)pkt_len) / std::max<uint64_t>(stride, 1u) + 1u;
            cap = std::min<uint64_t>(cap, std::max<uint64_t>(8u, ((uint64_t)n_pkt / 2048u) & ~7ull));
            cap = std::min<uint64_t>(cap, 64u);
            uint32_t* h_word = nullptr;
            uint32_t* d_word = nullptr;
            uint32_t tag = 0u, calls = 0u;
            uint32_t plan = d_off ? ring_plan(dev, d_base, reinterpret_cast<uint64_t>(d_off), 0xFFFFFFFFu, n_pkt,
                                              ip_ver, &h_word, &d_word, &tag, &calls)
                                  : ring_plan(dev, d_base, stride, pkt_len, n_pkt, ip_ver, &h_word, &d_word, &tag, &calls);
            if (d_word != nullptr) {
                a.plan = run0 | ((uint32_t)cap << 8) | (tag << 16);
                a.plan_out = d_word;
                if (plan == 0u && calls == 0u && plan_ahead(hs, n_pkt, kPlanAheadRing)) {
                    // the ring's first batch: its sampler alone, waited for
                    *reinterpret_cast<volatile uint32_t*>(h_word) = 0u;
                    NC_HIP(netcsum::launch_pkt_plan(a, ip_ver, hs));
                    plan = wait_plan_word(h_word, tag);
                    ahead_note = " ahead";
                }
                const uint32_t form = plan & 0x7u, pw = (plan >> 4) & 0xFu, prun = (plan >> 8) & 0xFFu;
                if (plan != 0u && d_off != nullptr) {
                    vl_wide = (plan & 8u) != 0u;
                    vl_inline = !vl_wide && ((plan >> 4) & 0xFu) != 0u;   // (the plan's reduced residency)
                }
                if (plan != 0u && form == 0u && run0 != 0u && prun == run0) {
                    bound = 0;
                    spw = run0;
                    plan_note = " plan=ring(form0)";
                } else if (plan != 0u && form == 2u && prun >= 1u && prun <= cap && (pw == 0u || (pw >= 3u && pw <= 8u))) {
                    bound = 2;
                    spw = prun;
                    a.res_waves = pw;
                    plan_note = pw ? (pw == 5u ? " plan=ring(live,5 waves)" : pw == 6u ? " plan=ring(live,6 waves)"
                                                                             : " plan=ring(live,waves)")
                                   : " plan=ring(live)";
                } else {
                    plan_note = " plan=first";
                }
            }
        }
        const bool snt = nt >= 0 ? (nt != 0) : true;
        // Tx passes: auto = two (8-B records, then a scatter pass: 1 M x 1500 B 0.2918 against 0.2954
        // ms in one pass) from 64 Ki datagrams up, one below (a burst is then a single launch)
        const int tp = g_tune_tx_passes.load();
        const bool two = tx && (rec_only != nullptr || tp == 2 || (tp == 0 && n_pkt >= 65536u));
        // IPv6 / mixed: the Rx and one-pass Tx kernels, and two-pass Tx's scatter pass, finish their
        // deferred datagrams themselves (no deferral word, no walk launch, no flags in scratch)
        if (bound >= 1 && d_off == nullptr) {          // (the device plan sizes its own runs)
            const uint64_t cap = (netcsum::kLiveReach - 128u - (uint64_t)pkt_len) / std::max<uint64_t>(stride, 1u) + 1u;
            if (spw > cap && tile > 0 && bound_default && dense) {
                bound = 0;                                // a run length asked for: the whole-span form
            } else {
                spw = (uint32_t)std::max<uint64_t>(1u, std::min<uint64_t>(spw, cap));
            }
        }
        char desc[208];
        snprintf(desc, sizeof desc, "pkt_stream_kernel<D=%d%s,%s,%s> block=256 pkts_per_wave=%u bound=%d%s%s%s%s%s", d,
                 snt ? ",nt" : "", tx ? "tx" : "rx", ip_ver == 4 ? "v4" : ip_ver == 6 ? "v6" : "mixed", spw, bound,
                 d_off ? (vl_inline ? " offlen (inline fallback)" : " offlen +pkt_vl_deferred_kernel") : "",
                 two ? " +pkt_scatter_kernel" : "", walk ? " +inline_v6_walk" : "", plan_note, ahead_note);
        netcsum::set_last_launch(desc);
        // scratch slot layout (one slot per (thread, device, stream), shared by every batch kind on the
        // stream, which stream order keeps apart): [0, 256) the words that must survive other calls'
        // data — +0 the lane-group walk pass's deferral word (tagged), +128 the varlen run word — then,
        // from +256, the records of two-pass Tx and, after them, offset/length batches' deferred-run list
        // (one index per run the stream kernel could not stream in order); the list's counters (count,
        // blocks done) are the slot's tail words, which the deferred pass leaves zero
        const size_t rec_bytes = (two && rec_only == nullptr) ? (size_t)n_pkt * sizeof(netcsum::PktTxRecord) : 0u;
        const size_t defer_bytes = (d_off && !vl_inline) ? (4u * (((size_t)n_pkt + spw - 1u) / spw) + 15u) & ~(size_t)15u : 0u;
        constexpr size_t kHdr = 256u;
        ScratchLease scratch;
        if (rec_bytes + defer_bytes) NC_HIP(scratch.acquire(dev, hs, kHdr + rec_bytes + defer_bytes));
        if (d_off && !vl_inline) {
            a.vl_list = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(scratch.ptr()) + kHdr + rec_bytes);
            a.vl_ctr = scratch.tail_words();
            a.vl_wide = vl_wide ? 1u : 0u;
        }
        netcsum::PktTxRecord* recs = rec_bytes ? reinterpret_cast<netcsum::PktTxRecord*>(static_cast<uint8_t*>(scratch.ptr()) + kHdr)
                                               : nullptr;
        if (rec_only != nullptr) {                        // zero-copy Tx burst: records only, no scatter
            NC_HIP(netcsum::launch_pkt_stream(a, ip_ver, d, spw, snt, tx, bound, hs, rec_only,
                                              false));
        } else {
            NC_HIP(netcsum::launch_pkt_stream(a, ip_ver, d, spw, snt, tx, bound, hs, two ? recs : nullptr));
        }
        if (a.vl_ctr != nullptr) scratch.tail_reset_enqueued();   // (launch_pkt_stream enqueued the deferred pass)
        NC_HIP(scratch.end());
        return NET_UTIL_ERR_NONE;
    }
    if (rec_only != nullptr) return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;   // (callers check the domain)
    a.tile = tile >= 0 ? (uint32_t)tile : (c.grid > 0 ? 0u : 2u);      // tile 2: best Rx/Tx point (r1m sweep)
    char desc[120];
    snprintf(desc, sizeof desc, "pkt_batch_kernel<G=%d,K=%d%s,%s,v%d> block=256 tile=%u%s", c.group_lanes,
             c.chunks_per_pass, c.nt ? ",nt" : "", tx ? "tx" : "rx", ip_ver, a.tile, walk ? " +pkt_v6_walk_kernel" : "");
    netcsum::set_last_launch(desc);
    ScratchLease scratch;                                 // [deferral word, 256 B | flags (own_flags)]
    if (walk) {
        NC_HIP(scratch.acquire(dev, hs, 256u + (own_flags ? n_pkt : 0u)));
        a.defer_word = static_cast<uint32_t*>(scratch.ptr());
        a.defer_tag = scratch.next_tag();
        if (own_flags) a.flags_out = static_cast<uint8_t*>(scratch.ptr()) + 256u;
    }
    NC_HIP(netcsum::launch_pkt_batch(a, c, tx, ip_ver, hs));
    if (walk) NC_HIP(netcsum::launch_pkt_v6_walk(a, tx, cu_count(dev), hs));
    NC_HIP(scratch.end());
    return NET_UTIL_ERR_NONE;
}

NET_ERR NetUtil_MI355X_ChkSumBatchChains(const void* d_base, const uint64_t* d_piece_off,
                                        const uint16_t* d_piece_len, const uint32_t* d_chain_first,
                                        const void* d_pseudo, uint32_t pseudo_stride, CPU_INT16U pseudo_len,
                                        uint32_t n_chains, void* d_out, NETCSUM_OP op, void* hip_stream) {
    if (op != NETCSUM_OP_DATA_CALC && op != NETCSUM_OP_DATA_VERIFY) return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
    if (n_chains == 0) return NET_UTIL_ERR_NONE;
    if (n_chains > 0x7FFFFFFFu) return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
    if (d_out == nullptr || d_chain_first == nullptr || d_piece_off == nullptr || d_piece_len == nullptr ||
        (d_pseudo == nullptr && pseudo_len != 0)) {
        return NET_ERR_FAULT_NULL_PTR;
    }
    int dev = 0;
    NC_HIP(hipGetDevice(&dev));
    netcsum::ChainBatchArgs a{};
    a.base = static_cast<const uint8_t*>(d_base);
    a.off = d_piece_off;
    a.len = d_piece_len;
    a.first = d_chain_first;
    a.pseudo = (pseudo_len != 0) ? static_cast<const uint8_t*>(d_pseudo) : nullptr;
    a.pseudo_stride = pseudo_stride;
    a.pseudo_len = pseudo_len;
    a.n = n_chains;
    a.verify = (op == NETCSUM_OP_DATA_VERIFY) ? 1u : 0u;
    a.out = d_out;
    // GROUP_LANES 16/32/64: chain_batch_kernel with that many lanes per chain; KERNEL 1: the
    // wave-per-chain kernel (4 chains per 256-thread block); otherwise (auto) the two-pass form
    // (per-piece sums in piece order, then a combine pass per chain), its records in this thread's
    // scratch for this stream: room for max(2^20, 128 x chains) pieces (a batch with more pieces is
    // done by the wave-per-chain form inside the combine pass).
    int g = g_tune_group.load();
    g = (g == 16 || g == 32 || g == 64) ? g : 0;
    // The records are capped at 2^24 pieces (128 MiB per thread and stream): a larger batch runs its
    // pieces past the cap in the wave-per-chain form inside pass 1, and a thread whose scratch cannot
    // be allocated (or is pinned by a stream capture) takes the wave-per-chain kernel instead.
    if (g == 0 && g_tune_kernel.load() != 1) {
        const uint64_t cap = std::min<uint64_t>(std::max<uint64_t>(1ull << 20, 128ull * n_chains), 1ull << 24);
        const int kern = g_tune_kernel.load();
        // the default (0) and 5: one record per piece (4 B); 3 the round-5 live form, others the tiled
        // 16-lane groups (both 8 B per piece)
        const bool one_rec = kern == 0 || kern == 5;
        ScratchLease scratch;
        if (scratch.acquire(dev, static_cast<hipStream_t>(hip_stream), (size_t)cap * (one_rec ? 4u : 8u)) == hipSuccess) {
            // pass 1: tiled 16-lane groups, or with TUNE_KERNEL 3 the live-sector stream in runs of 16
            // pieces (TUNE_TILE 1..64 sets the run, TUNE_CHUNKS 4 the depth) — 0.1993-0.2046 ms on the
            // chain row against 0.1756-0.1803 for the groups (profiles/r5v_chains.log: two wave totals
            // per piece end, the byte and the half-word sums, cost more than the sectors save there)
            // Default / TUNE_KERNEL 5 (round 6): the segment live-sector stream with ONE wave total per piece
            // end, the piece's half-word sum, combined modulo 65535 (chain_combine_h_kernel)
            const int tk = g_tune_tile.load(), ch = g_tune_chunks.load();
            // runs: TUNE_TILE, else 16 pieces (round 5's live form) / 12 (the one-record form: 0.1686-0.1691
            // ms on the chain row against 0.1709-0.1715 for 16, profiles/r6v_*, r6w_*)
            const uint32_t live = (kern != 3 && !one_rec) ? 0u : (tk >= 1 && tk <= 64) ? (uint32_t)tk : one_rec ? 12u : 16u;
            const int depth = ch == 4 ? 4 : 8;
            char d[128];
            if (one_rec) {
                const bool cmp = netcsum::live_compact();
                const int cl = g_tune_chain_combine.load() == 64 ? 64 : 16;
                snprintf(d, sizeof d, "seg_live_varlen_kernel<D=%d,chain,nt%s> pieces_per_wave=%u +chain_combine_h_kernel<%d>",
                         depth, cmp ? ",compact" : "", live, cl);
                netcsum::set_last_launch(d);
                NC_HIP(netcsum::launch_chain_two_pass_h(a, static_cast<uint32_t*>(scratch.ptr()), (uint32_t)cap, cu_count(dev),
                                                        static_cast<hipStream_t>(hip_stream), live, depth, cmp, cl));
                NC_HIP(scratch.end());
                return NET_UTIL_ERR_NONE;
            }
            if (live) {
                snprintf(d, sizeof d, "chain_live_piece_kernel<D=%d,nt> pieces_per_wave=%u +chain_combine_kernel", depth, live);
            } else {
                snprintf(d, sizeof d, "chain_piece_kernel<G=16,K=6,tile=64,nt> +chain_combine_kernel");
            }
            netcsum::set_last_launch(d);
            NC_HIP(netcsum::launch_chain_two_pass(a, static_cast<uint64_t*>(scratch.ptr()), (uint32_t)cap, cu_count(dev),
                                                  static_cast<hipStream_t>(hip_stream), live, depth));
            NC_HIP(scratch.end());
            return NET_UTIL_ERR_NONE;
        }
        (void)hipGetLastError();                          // a failed allocation is not this launch's error
    }
    netcsum::set_last_launch(g ? "chain_batch_kernel" : "chain_wave_kernel");
    const uint32_t gpb = g ? 256u / (uint32_t)g : 4u;
    const uint64_t need = ((uint64_t)n_chains + gpb - 1u) / gpb;
    int grid = g_tune_grid.load();
    if (grid <= 0) grid = (int)std::min<uint64_t>(need, (uint64_t)cu_count(dev) * (g ? 16u : 64u));
    NC_HIP(netcsum::launch_chain_batch(a, g, grid, static_cast<hipStream_t>(hip_stream)));
    return NET_UTIL_ERR_NONE;
}

NET_ERR NetUtil_MI355X_RxValidateIPv4(const void* d_base, const uint64_t* d_off, const uint16_t* d_len,
                                      uint64_t stride, CPU_INT16U pkt_len, uint32_t n_pkt, uint8_t* d_flags,
                                      void* hip_stream) {
    return pkt_batch(d_base, d_off, d_len, stride, pkt_len, n_pkt, d_flags, 1, false, 4, hip_stream);
}

NET_ERR NetUtil_MI355X_TxFinalizeIPv4(void* d_base, const uint64_t* d_off, const uint16_t* d_len, uint64_t stride,
                                      CPU_INT16U pkt_len, uint32_t n_pkt, uint8_t* d_flags, int udp_tx_csum,
                                      void* hip_stream) {
    return pkt_batch(d_base, d_off, d_len, stride, pkt_len, n_pkt, d_flags, udp_tx_csum ? 1u : 0u, true, 4, hip_stream);
}

NET_ERR NetUtil_MI355X_RxValidateIPv6(const void* d_base, const uint64_t* d_off, const uint16_t* d_len,
                                      uint64_t stride, CPU_INT16U pkt_len, uint32_t n_pkt, uint8_t* d_flags,
                                      void* hip_stream) {
    return pkt_batch(d_base, d_off, d_len, stride, pkt_len, n_pkt, d_flags, 1, false, 6, hip_stream);
}

NET_ERR NetUtil_MI355X_RxValidateIP(const void* d_base, const uint64_t* d_off, const uint16_t* d_len,
                                    uint64_t stride, CPU_INT16U pkt_len, uint32_t n_pkt, uint8_t* d_flags,
                                    void* hip_stream) {
    return pkt_batch(d_base, d_off, d_len, stride, pkt_len, n_pkt, d_flags, 1, false, 0, hip_stream);
}

NET_ERR NetUtil_MI355X_TxFinalizeIPv6(void* d_base, const uint64_t* d_off, const uint16_t* d_len, uint64_t stride,
                                      CPU_INT16U pkt_len, uint32_t n_pkt, uint8_t* d_flags, int udp_tx_csum,
                                      void* hip_stream) {
    return pkt_batch(d_base, d_off, d_len, stride, pkt_len, n_pkt, d_flags, udp_tx_csum ? 1u : 0u, true, 6, hip_stream);
}

NET_ERR NetUtil_MI355X_TxFinalizeIP(void* d_base, const uint64_t* d_off, const uint16_t* d_len, uint64_t stride,
                                    CPU_INT16U pkt_len, uint32_t n_pkt, uint8_t* d_flags, int udp_tx_csum,
                                    void* hip_stream) {
    return pkt_batch(d_base, d_off, d_len, stride, pkt_len, n_pkt, d_flags, udp_tx_csum ? 1u : 0u, true, 0, hip_stream);
}

// Burst adapters of the reference's checksum-offload seam (include/netcsum_mi355x.h (2b'')): the mixed
// IPv4 / IPv6 kernels with the action written beside each verdict (Rx) and the per-datagram UDP policy
// of the offload's 0xFFFF placeholder (Tx).
NET_ERR NetUtil_MI355X_RxBurst(const void* d_base, const uint64_t* d_off, const uint16_t* d_len, uint64_t stride,
                               CPU_INT16U pkt_len, uint32_t n_pkt, uint32_t rx_cfg, uint8_t* d_action, uint8_t* d_flags,
                               void* hip_stream) {
    if (n_pkt != 0 && d_action == nullptr) return NET_ERR_FAULT_NULL_PTR;
    if (rx_cfg & ~(uint32_t)NETCSUM_RXCFG_UDP_DISCARD_NO_CHK_SUM) return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
    return pkt_batch(d_base, d_off, d_len, stride, pkt_len, n_pkt, d_flags, 1u, false, 0, hip_stream, d_action, rx_cfg);
}

uint8_t NetUtil_MI355X_RxAction(uint8_t flags, uint8_t proto, int ipv6, uint32_t rx_cfg) {
    return (uint8_t)netcsum::rx_action(flags, proto, ipv6 != 0, rx_cfg);
}

NET_ERR NetUtil_MI355X_TxBurst(void* d_base, const uint64_t* d_off, const uint16_t* d_len, uint64_t stride,
                               CPU_INT16U pkt_len, uint32_t n_pkt, uint8_t* d_flags, void* hip_stream) {
    return pkt_batch(d_base, d_off, d_len, stride, pkt_len, n_pkt, d_flags, 2u, true, 0, hip_stream);
}

// ----------------------------------------------------------- host-memory batches (PCIe-inclusive)
// The path starts and ends in host memory (NIC Rx buffers, IF/net_if.c:6593; socket Tx buffers,
// Source/net_sock.c:5531). Each entry point below is its device form run over chunks on the three
// pipeline streams of the calling thread's context: chunk k's bytes [lo, hi) go H2D (with its
// descriptors rebased to lo, staged in pinned memory), the device form runs on the copy, its results
// come D2H — and for Tx the chunk's bytes themselves, written back over [lo, hi) of the caller's
// buffer — while chunks k +- 1 copy and compute on the other streams. Slot k mod 3 is reused after its
// stream has drained it. Host buffers should be pinned (hipHostMalloc / hipHostRegister) for the
// copies to overlap; the call returns when every output is in host memory.

NET_ERR NetUtil_MI355X_ChkSumBatchVarLenHost(const void* h_base, const uint64_t* h_seg_off, const uint16_t* h_seg_len,
                                             const void* h_pseudo, uint32_t pseudo_stride, CPU_INT16U pseudo_len,
                                             uint32_t n_seg, void* h_out, NETCSUM_OP op, uint32_t n_chunks) {
    NET_ERR e = check_op(op, h_pseudo, pseudo_len);
    if (e != NET_UTIL_ERR_NONE) return e;
    if (n_seg == 0) return NET_UTIL_ERR_NONE;
    if (n_seg > 0x7FFFFFFFu) return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
    if (h_out == nullptr || h_base == nullptr || h_seg_off == nullptr || h_seg_len == nullptr) return NET_ERR_FAULT_NULL_PTR;
    HostCtx* cp = nullptr;
    e = host_ctx(&cp);
    if (e != NET_UTIL_ERR_NONE) return e;
    HostCtx& c = *cp;
    const bool verify = (op == NETCSUM_OP_DATA_VERIFY || op == NETCSUM_OP_HDR_VERIFY);
    const size_t elt = verify ? 1u : 2u;
    const bool has_ph = h_pseudo != nullptr && pseudo_len != 0;
    std::vector<HostChunk> ch;
    const uint64_t maxb = plan_chunks(h_seg_off, h_seg_len, 0, 0, n_seg, n_chunks, ch);
    const uint32_t per = ch[0].ns;
    const size_t ph_bytes = has_ph ? (size_t)(per - 1u) * pseudo_stride + pseudo_len : 0u;
    // device slot: [bytes | offsets | lengths | pseudo-headers | outputs]; host slot: [offsets | lengths]
    const size_t o_off = al256(maxb), o_len = o_off + al256((size_t)per * 8u), o_ph = o_len + al256((size_t)per * 2u);
    const size_t o_out = o_ph + al256(ph_bytes), dev_need = o_out + al256((size_t)per * elt);
    e = ensure_pipe(c, dev_need, al256((size_t)per * 8u) + (size_t)per * 2u);
    if (e != NET_UTIL_ERR_NONE) return e;
    PipeDrainOnExit guard{c};
    for (size_t k = 0; k < ch.size(); ++k) {
        const HostChunk& q = ch[k];
        const int j = (int)(k % 3u);
        hipStream_t st = c.pstream[j];
        if (k >= 3) NC_HIP(hipStreamSynchronize(st));       // slot j's staging is free again
        uint8_t* d = c.d_pipe[j];
        uint64_t* h_o = reinterpret_cast<uint64_t*>(c.h_pipe[j]);
        uint16_t* h_l = reinterpret_cast<uint16_t*>(c.h_pipe[j] + al256((size_t)per * 8u));
        for (uint32_t i = 0; i < q.ns; ++i) {
            h_o[i] = h_seg_off[q.s0 + i] - q.lo;
            h_l[i] = h_seg_len[q.s0 + i];
        }
        NC_HIP(hipMemcpyAsync(d, static_cast<const uint8_t*>(h_base) + q.lo, q.hi - q.lo, hipMemcpyHostToDevice, st));
        NC_HIP(hipMemcpyAsync(d + o_off, h_o, (size_t)q.ns * 8u, hipMemcpyHostToDevice, st));
        NC_HIP(hipMemcpyAsync(d + o_len, h_l, (size_t)q.ns * 2u, hipMemcpyHostToDevice, st));
        if (has_ph) {
            NC_HIP(hipMemcpyAsync(d + o_ph, static_cast<const uint8_t*>(h_pseudo) + (size_t)q.s0 * pseudo_stride,
                                  (size_t)(q.ns - 1u) * pseudo_stride + pseudo_len, hipMemcpyHostToDevice, st));
        }
        netcsum::SegBatchArgs a{};
        a.base = d;
        a.seg_off = reinterpret_cast<const uint64_t*>(d + o_off);
        a.seg_len_v = reinterpret_cast<const uint16_t*>(d + o_len);
        a.pseudo = has_ph ? d + o_ph : nullptr;
        a.pseudo_stride = pseudo_stride;
        a.pseudo_len = has_ph ? pseudo_len : 0u;
        a.n_seg = q.ns;
        a.verify = verify ? 1u : 0u;
        a.out = d + o_out;
        // (a segment's byte parity is taken from the device address it is read at, so the copy's new
        // alignment changes nothing)
        e = launch_batch(a, 0u, st);
        if (e != NET_UTIL_ERR_NONE) return e;
        NC_HIP(hipMemcpyAsync(static_cast<uint8_t*>(h_out) + (size_t)q.s0 * elt, d + o_out, (size_t)q.ns * elt,
                              hipMemcpyDeviceToHost, st));
    }
    for (int j = 0; j < 3; ++j) NC_HIP(hipStreamSynchronize(c.pstream[j]));
    guard.done = true;
    return NET_UTIL_ERR_NONE;
}

// ---- zero-copy bursts (NetUtil_MI355X_RxBurstHost / RxValidateIPHost up to kBurstZC frames)
// A driver's burst is a few to a few hundred frames (the template's Rx ring holds 10 buffers,
// Cfg/Template/net_dev_cfg.c:147), so its cost is fixed, not bandwidth: an H2D copy, a launch, a D2H
// copy and a stream synchronisation took 19.3 us for one frame (profiles/r3x_burst_latency.jsonl).
// When the caller's ring is pinned (device-accessible host memory) the kernel reads it in place over
// PCIe, and its flags and actions (Tx: 8-B field records) go straight into coherent pinned memory that
// the host set to a sentinel no result can take (0xFF); the host polls them until every one has
// arrived — each is written once, so no completion protocol is needed — instead of synchronising a
// stream. By default (TUNE_BURST_ZERO_COPY 3) the kernel is this thread's resident burst server
// (burst_server_run below), which takes each burst from a posted line: no launch per burst.
// TUNE_BURST_ZERO_COPY 2: a launch per burst; 1: the results go to device memory and a one-wave
// completion kernel copies them into coherent memory, then stores a tagged completion word
// (system-scope release after the wave's own stores) that the host polls. tools/burst_latency.c zc,
// profiles/r4k_burst_zc.jsonl: 1 / 64 frames 6.9 / 11.2 us (3), 10.8 / 12.9 us (2), 12.7 / 15.1 us
// (1). A pageable ring takes the copy path.
constexpr uint32_t kBurstZC = 4096u;                    // frames
// Over PCIe a burst is latency-bound: the whole-slot stream (bound 0) issues the pieces with the
// parse's loads (one round trip) where the live-piece forms parse first (two); it applies to
// strided rings with gaps <= 64 B, the others keep the default (tools/burst_latency.c zc,
// profiles/r4k_burst_zc.jsonl: a launch per burst, 64 frames 12.9 us against 13.9 us in form 2)
constexpr int kBurstBound = 0;
constexpr uint64_t kBurstZCSpan = 64ull << 20;          // ring bytes the kernel may read in place
constexpr size_t kBurstWord = 0, kBurstPost = 64, kBurstClosed = 128, kBurstFlags = 256, kBurstAct = kBurstFlags + kBurstZC,
                 kBurstOff = kBurstAct + kBurstZC, kBurstLen = kBurstOff + 8u * kBurstZC,
                 kBurstRec = kBurstLen + 2u * kBurstZC, kBurstHostBytes = kBurstRec + 8u * kBurstZC;
// device side: [flags | actions | Tx records]
constexpr size_t kBurstDevRec = 2u * kBurstZC, kBurstDevBytes = kBurstDevRec + 8u * kBurstZC;

// The device address of host bytes [h, h + span) when they are one pinned (device-mapped) host
// allocation, else nullptr.
static const uint8_t* pinned_alias(const void* h, uint64_t span) {
    if (h == nullptr || span == 0) return nullptr;
    hipPointerAttribute_t a0{}, a1{};
    const uint8_t* last = static_cast<const uint8_t*>(h) + (span - 1u);
    if (hipPointerGetAttributes(&a0, h) != hipSuccess || hipPointerGetAttributes(&a1, last) != hipSuccess) {
        (void)hipGetLastError();                        // pageable memory: not an error of this call
        return nullptr;
    }
    if (a0.type != hipMemoryTypeHost || a1.type != hipMemoryTypeHost || a0.devicePointer == nullptr ||
        static_cast<const uint8_t*>(a1.devicePointer) != static_cast<const uint8_t*>(a0.devicePointer) + (span - 1u)) {
        return nullptr;
    }
    return static_cast<const uint8_t*>(a0.devicePointer);
}

static NET_ERR ensure_burst(HostCtx& c) {
    if (c.h_burst != nullptr) return NET_UTIL_ERR_NONE;
    NC_HIP(hipMalloc(&c.d_burst, kBurstDevBytes));
    NC_HIP(hipHostMalloc(&c.h_burst, kBurstHostBytes, hipHostMallocMapped | hipHostMallocCoherent));
    NC_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&c.h_burst_dev), c.h_burst, 0));
    return NET_UTIL_ERR_NONE;
}

// Polls the completion word of tag (2 s, then a stream synchronisation reports a failed launch).
static NET_ERR burst_wait(HostCtx& c, uint32_t tag) {
    volatile unsigned long long* w = reinterpret_cast<volatile unsigned long long*>(c.h_burst + kBurstWord);
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spin = 0; (uint32_t)*w != tag; ++spin) {
        if ((spin & 1023u) == 1023u && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
            NC_HIP(hipStreamSynchronize(c.stream));
            if ((uint32_t)*w != tag) return dev_fail("burst completion word", hipErrorUnknown);
            break;
        }
    }
    return NET_UTIL_ERR_NONE;
}

// Polls until ready(i) holds for every i < n (each result is written once by the kernel, into
// coherent memory initialised to a sentinel), scanning forward; after 2 s a stream synchronisation
// reports a failed launch.
extern "C++" {
template <class Ready>
static NET_ERR burst_poll(HostCtx& c, Ready ready, uint32_t n) {
    const auto t0 = std::chrono::steady_clock::now();
    uint32_t i = 0, spin = 0;
    while (i < n) {
        if (ready(i)) {
            ++i;
            continue;
        }
        if ((++spin & 1023u) == 0u && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
            NC_HIP(hipStreamSynchronize(c.stream));
            for (; i < n; ++i) {
                if (!ready(i)) return dev_fail("burst results", hipErrorUnknown);
            }
        }
    }
    return NET_UTIL_ERR_NONE;
}

// ---- resident burst server (TUNE_BURST_ZERO_COPY 3; netcsum_pktstream.hip burst_server_kernel)
// A launch per burst is most of a small burst's cost (launch, dispatch, then the kernel's PCIe round
// trips). This context's server is launched on a stream of its own and serves every burst posted to
// it until it has been idle for TUNE_BURST_SERVER_IDLE_US (default 500 us: a device-wide
// synchronisation waits at most that long for it after the last burst) or resident for
// TUNE_BURST_SERVER_LIFE_US (default 1000 us) even while bursts keep coming: HIP maps the process's
// streams onto GPU_MAX_HW_QUEUES hardware queues, and kernels of a stream sharing the server's queue
// wait behind it, so each launch is bounded and the next burst relaunches it (one launch per ms of
// continuous service). Posting: the line's fields,
// then its burst number (a read that sees the new number with stale fields fails the check), a
// full fence, then the blocks' closed marks — a block that closed may have missed the post
// (Dekker's handshake, see the kernel), so the host waits the server out and relaunches it if the
// burst is not served. A server that stopped unnoticed is found by a stream query after 200 us
// without results.
// 16 blocks x 4 waves: a block's leader polls the post line (16 64-B reads per poll round); 4 blocks
// of 16 waves were slower from 10 frames up (tools/burst_latency.c, 64 frames 14.8 us against 13.1 us
// for a launch per burst: 16 waves on one CU queue their PCIe reads)
constexpr int kServerBlocks = 16;
static_assert(kServerBlocks <= netcsum::kBurstServerMaxBlocks && kBurstClosed + 8u * kServerBlocks <= kBurstFlags,
              "closed marks");

static void write_post(HostCtx& c, const netcsum::BurstPost& p) {
    volatile uint32_t* l = reinterpret_cast<volatile uint32_t*>(c.h_burst + kBurstPost);
    const uint32_t* q = reinterpret_cast<const uint32_t*>(&p);
    for (int i = 2; i < 16; ++i) l[i] = q[i];            // fields, check
    std::atomic_thread_fence(std::memory_order_release);
    *reinterpret_cast<volatile uint64_t*>(c.h_burst + kBurstPost) = p.seq;
    std::atomic_thread_fence(std::memory_order_seq_cst); // the post before the closed marks are read
}

static NET_ERR launch_server(HostCtx& c, uint64_t seq0) {
    volatile unsigned long long* closed = reinterpret_cast<volatile unsigned long long*>(c.h_burst + kBurstClosed);
    for (int b = 0; b < kServerBlocks; ++b) closed[b] = 0ull;
    int khz = 0;
    NC_HIP(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c.dev));
    netcsum::BurstServerArgs a{};
    a.post = reinterpret_cast<const netcsum::BurstPost*>(c.h_burst_dev + kBurstPost);
    a.closed = reinterpret_cast<unsigned long long*>(c.h_burst_dev + kBurstClosed);
    a.flags = c.h_burst_dev + kBurstFlags;
    a.act = c.h_burst_dev + kBurstAct;
    a.rec = reinterpret_cast<netcsum::PktTxRecord*>(c.h_burst_dev + kBurstRec);
    a.off = reinterpret_cast<const uint64_t*>(c.h_burst_dev + kBurstOff);
    a.len = reinterpret_cast<const uint16_t*>(c.h_burst_dev + kBurstLen);
    a.seq0 = seq0;
    a.idle_ticks = (uint64_t)std::max(1, g_tune_burst_idle.load()) * (uint64_t)std::max(khz, 1) / 1000u;
    a.life_ticks = (uint64_t)std::max(1, g_tune_burst_life.load()) * (uint64_t)std::max(khz, 1) / 1000u;
    NC_HIP(netcsum::launch_burst_server(a, kServerBlocks, c.sstream));
    c.server_live = true;
    return NET_UTIL_ERR_NONE;
}

// Waits for the server's stream for at most limit_ms (a stream query loop, never a blocking
// synchronisation): a server launch queued behind other work on its hardware queue still ends, since
// every launch of every server is bounded by its residency limit, but the caller's wait must not
// depend on that. hipErrorNotReady when the stream is still busy at the deadline: a burst whose server
// is still queued 2 s after its post (burst_server_run's wait_out) fails with NET_UTIL_ERR_MI355X_DEV,
// and the server stays marked live (it still serves or stops). The first 20 us poll back to back (a
// server leaves within one burst of its stop), after that each poll yields the host core.
static hipError_t server_stream_wait(hipStream_t s, int limit_ms) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        const hipError_t e = hipStreamQuery(s);
        const auto el = std::chrono::steady_clock::now() - t0;
        if (e != hipErrorNotReady || el > std::chrono::milliseconds(limit_ms)) {
            return e;
        }
        if (el > std::chrono::microseconds(20)) std::this_thread::yield();
    }
}

// Posts the stop line and waits for the server: limit_ms 0 without limit (release(), which frees the
// memory the server reads), else at most limit_ms; false if the server is still queued or running
// then (server_live stays set: it will serve whatever is posted next, or stop).
bool HostCtx::stop_server(int limit_ms) {
    if (server_live && sstream && h_burst) {
        netcsum::BurstPost p{};
        p.seq = netcsum::kBurstStop;
        p.check = netcsum::burst_post_check(p);
        write_post(*this, p);
        if (limit_ms <= 0) {
            (void)hipStreamSynchronize(sstream);
        } else if (server_stream_wait(sstream, limit_ms) == hipErrorNotReady) {
            return false;
        }
    }
    server_live = false;
    return true;
}

template <class Ready>
static NET_ERR burst_server_run(HostCtx& c, netcsum::BurstPost p, Ready ready, uint32_t n) {
    if (c.sstream == nullptr) NC_HIP(hipStreamCreateWithFlags(&c.sstream, hipStreamNonBlocking));
    auto all_ready = [&](uint32_t from) {
        for (uint32_t i = from; i < n; ++i) {
            if (!ready(i)) return false;
        }
        return true;
    };
    auto wait_out = [&](uint32_t from) -> NET_ERR {     // the server has stopped, or is stopping
        NC_HIP(server_stream_wait(c.sstream, 2000));    // (its blocks stop together, after one burst at most)
        c.server_live = false;
        return all_ready(from) ? NET_UTIL_ERR_NONE : launch_server(c, p.seq - 1u);
    };
    p.seq = ++c.post_seq;
    p.check = netcsum::burst_post_check(p);
    write_post(c, p);
    NET_ERR e = NET_UTIL_ERR_NONE;
    if (!c.server_live) {
        e = launch_server(c, p.seq - 1u);
    } else {
        const volatile unsigned long long* closed =
            reinterpret_cast<const volatile unsigned long long*>(c.h_burst + kBurstClosed);
        bool any = false;
        for (int b = 0; b < kServerBlocks; ++b) any = any || closed[b] != 0ull;
        if (any) e = wait_out(0u);
    }
    if (e != NET_UTIL_ERR_NONE) return e;
    const auto t0 = std::chrono::steady_clock::now();
    auto t_check = t0 + std::chrono::microseconds(200);
    uint32_t i = 0, spin = 0;
    while (i < n) {
        if (ready(i)) {
            ++i;
            continue;
        }
        if ((++spin & 255u) != 0u) continue;
        const auto t = std::chrono::steady_clock::now();
        if (t < t_check) continue;
        t_check = t + std::chrono::microseconds(200);
        if (c.server_live && hipStreamQuery(c.sstream) == hipSuccess) {   // stopped without serving it
            e = wait_out(i);
            if (e != NET_UTIL_ERR_NONE) return e;
        } else if (t - t0 > std::chrono::seconds(2)) {
            if (!c.stop_server(2000)) return dev_fail("burst server still queued or running", hipErrorNotReady);
            if (!all_ready(i)) return dev_fail("burst server results", hipErrorUnknown);
        }
    }
    return NET_UTIL_ERR_NONE;
}

// NetUtil_MI355X_LastLaunch after a zero-copy burst: which path served it (the tests check that the
// zero-copy path, not the copy pipeline, was taken)
static void server_launch_name(uint32_t form, uint32_t spw, bool tx) {
    char d[96];
    snprintf(d, sizeof d, "burst_server_kernel %s form=%s pkts_per_wave=%u zero-copy", tx ? "tx" : "rx",
             form == netcsum::kBurstWhole ? "whole" : form == netcsum::kBurstLive ? "live" : "offlen", spw);
    netcsum::set_last_launch(d);
}

static void mark_zero_copy_launch(int zc) {
    char d[200];
    snprintf(d, sizeof d, "%s zero-copy%s", NetUtil_MI355X_LastLaunch(), zc == 1 ? " +burst_done_kernel" : "");
    netcsum::set_last_launch(d);
}

// The server's form for a burst (BurstPost::form >> 1 and its run length), or false when the burst is
// outside the run-stream kernel's domain (the launch path takes it).
static bool server_form(const uint64_t* h_off, uint64_t stride, CPU_INT16U pkt_len, uint32_t n_pkt, uint32_t* form,
                        uint32_t* spw) {
    netcsum::PktBatchArgs a{};
    a.off = h_off;
    a.len = reinterpret_cast<const uint16_t*>(h_off);     // (only tested against nullptr)
    a.stride = stride;
    a.len_u = pkt_len;
    a.n = n_pkt;
    uint32_t run = std::max<uint32_t>(1u, std::min<uint32_t>(16u, (n_pkt + 4u * kServerBlocks - 1u) / (4u * kServerBlocks)));
    if (h_off != nullptr) {
        *form = netcsum::kBurstOffLen;
        if (!netcsum::pkt_stream_supported(a, 0, 2)) return false;
    } else if (stride <= (uint64_t)pkt_len + 64u && netcsum::pkt_stream_supported(a, 0, 0)) {
        *form = netcsum::kBurstWhole;                   // (kBurstBound: one PCIe round trip)
    } else if (netcsum::pkt_stream_supported(a, 0, 2)) {
        *form = netcsum::kBurstLive;
        const uint64_t cap = (netcsum::kLiveReach - 128u - (uint64_t)pkt_len) / std::max<uint64_t>(stride, 1u) + 1u;
        run = (uint32_t)std::max<uint64_t>(1u, std::min<uint64_t>(run, cap));
    } else {
        return false;
    }
    *spw = run;
    return true;
}
}  // extern "C++"

// Rx over a pinned ring in place. *taken = false: the burst does not qualify (the caller takes the
// copy path); else the call's result.
static NET_ERR rx_burst_zero_copy(HostCtx& c, const void* h_base, const uint64_t* h_off, const uint16_t* h_len,
                                  uint64_t stride, CPU_INT16U pkt_len, uint32_t n_pkt, uint8_t* h_flags,
                                  uint8_t* h_action, uint32_t rx_cfg, bool* taken) {
    *taken = false;
    if (n_pkt > kBurstZC) return NET_UTIL_ERR_NONE;
    uint64_t span = 0;
    if (h_off == nullptr) {
        span = (uint64_t)(n_pkt - 1u) * stride + pkt_len;
    } else {
        for (uint32_t i = 0; i < n_pkt; ++i) span = std::max<uint64_t>(span, h_off[i] + h_len[i]);
    }
    if (span > kBurstZCSpan) return NET_UTIL_ERR_NONE;
    const uint8_t* d_ring = pinned_alias(h_base, span);
    if (d_ring == nullptr) return NET_UTIL_ERR_NONE;
    *taken = true;
    NET_ERR e = ensure_burst(c);
    if (e != NET_UTIL_ERR_NONE) return e;
    const uint64_t* d_off = nullptr;
    const uint16_t* d_len = nullptr;
    if (h_off != nullptr) {                             // descriptors: staged in coherent pinned memory
        std::memcpy(c.h_burst + kBurstOff, h_off, (size_t)n_pkt * 8u);
        std::memcpy(c.h_burst + kBurstLen, h_len, (size_t)n_pkt * 2u);
        d_off = reinterpret_cast<const uint64_t*>(c.h_burst_dev + kBurstOff);
        d_len = reinterpret_cast<const uint16_t*>(c.h_burst_dev + kBurstLen);
    }
    uint32_t form = 0, spw = 0;
    const int zc = g_tune_burst_zc.load();
    if (zc == 3 && server_form(h_off, stride, pkt_len, n_pkt, &form, &spw)) {   // the resident server
        uint8_t* hf = c.h_burst + kBurstFlags;
        uint8_t* ha = c.h_burst + kBurstAct;
        std::memset(hf, 0xFF, n_pkt);
        std::memset(ha, 0xFF, n_pkt);
        netcsum::BurstPost p{};
        p.ring = reinterpret_cast<uint64_t>(d_ring);
        p.stride = (uint32_t)stride;
        p.n = n_pkt;
        p.pkt_len = pkt_len;
        p.spw = spw;
        p.form = form << 1;
        p.rx_cfg = rx_cfg;
        server_launch_name(form, spw, false);
        e = burst_server_run(c, p, [&](uint32_t i) { return *(volatile uint8_t*)(hf + i) != 0xFFu &&
                                                            *(volatile uint8_t*)(ha + i) != 0xFFu; }, n_pkt);
        if (e != NET_UTIL_ERR_NONE) return e;
        if (h_flags) std::memcpy(h_flags, hf, n_pkt);
        if (h_action) std::memcpy(h_action, ha, n_pkt);
        return NET_UTIL_ERR_NONE;
    }
    if (zc >= 2) {                                      // results straight into coherent memory, polled
        uint8_t* hf = c.h_burst + kBurstFlags;
        uint8_t* ha = c.h_burst + kBurstAct;
        std::memset(hf, 0xFF, n_pkt);                   // sentinels: no flag byte or action is 0xFF
        std::memset(ha, 0xFF, n_pkt);
        e = pkt_batch(d_ring, d_off, d_len, stride, pkt_len, n_pkt, c.h_burst_dev + kBurstFlags, 1u, false, 0, c.stream,
                      c.h_burst_dev + kBurstAct, rx_cfg, nullptr, nullptr, kBurstBound);
        if (e != NET_UTIL_ERR_NONE) return e;
        mark_zero_copy_launch(2);
        e = burst_poll(c, [&](uint32_t i) { return *(volatile uint8_t*)(hf + i) != 0xFFu &&
                                                   *(volatile uint8_t*)(ha + i) != 0xFFu; }, n_pkt);
        if (e != NET_UTIL_ERR_NONE) return e;
        if (h_flags) std::memcpy(h_flags, hf, n_pkt);
        if (h_action) std::memcpy(h_action, ha, n_pkt);
        return NET_UTIL_ERR_NONE;
    }
    uint8_t* d_fl = c.d_burst;
    uint8_t* d_act = h_action ? c.d_burst + kBurstZC : nullptr;
    e = pkt_batch(d_ring, d_off, d_len, stride, pkt_len, n_pkt, d_fl, 1u, false, 0, c.stream, d_act, rx_cfg, nullptr,
                  nullptr, kBurstBound);
    if (e != NET_UTIL_ERR_NONE) return e;
    mark_zero_copy_launch(1);
    if (++c.seq == 0u) c.seq = 1u;
    const uint32_t tag = c.seq;
    *reinterpret_cast<volatile unsigned long long*>(c.h_burst + kBurstWord) = 0ull;
    NC_HIP(netcsum::launch_burst_done(d_fl, d_act, n_pkt, c.h_burst_dev + kBurstFlags, c.h_burst_dev + kBurstAct,
                                      reinterpret_cast<unsigned long long*>(c.h_burst_dev + kBurstWord), tag, c.stream));
    e = burst_wait(c, tag);
    if (e != NET_UTIL_ERR_NONE) return e;
    if (h_flags) std::memcpy(h_flags, c.h_burst + kBurstFlags, n_pkt);
    if (h_action) std::memcpy(h_action, c.h_burst + kBurstAct, n_pkt);
    return NET_UTIL_ERR_NONE;
}

static NET_ERR pkt_host_copy(void* h_base, const uint64_t* h_off, const uint16_t* h_len, uint64_t stride,
                             CPU_INT16U pkt_len, uint32_t n_pkt, uint8_t* h_flags, uint8_t* h_action, uint32_t rx_cfg,
                             uint32_t udp_mode, bool tx, uint32_t n_chunks);

// Tx over a pinned ring: the checksum pass reads the ring in place and writes one 8-B
// record per datagram (PktTxRecord) to device memory — never into the ring —, the completion kernel
// copies the records into coherent pinned memory, and the host writes the fields into its ring (as
// the copy pipeline's gather records do). Datagrams whose IPv6 extension chain runs past the
// kernel's window (flag EXT_HDR: walked by a later pass in the device forms) are finished by the copy
// path afterwards, as an offset/length batch of just those datagrams. *taken as for Rx.
static NET_ERR tx_burst_zero_copy(HostCtx& c, void* h_base, const uint64_t* h_off, const uint16_t* h_len,
                                  uint64_t stride, CPU_INT16U pkt_len, uint32_t n_pkt, uint8_t* h_flags,
                                  uint32_t udp_mode, bool* taken) {
    *taken = false;
    if (n_pkt > kBurstZC || g_tune_kernel.load() == 2) return NET_UTIL_ERR_NONE;
    netcsum::PktBatchArgs a{};
    a.stride = stride;
    a.len_u = pkt_len;
    a.n = n_pkt;
    a.off = h_off;                                      // (only tested against nullptr here)
    a.len = h_len;
    // the records come from the run-stream kernel only: the burst qualifies where pkt_batch picks it
    // (the tuned bound, else the whole-span form 0 or the live-piece form 2), and the server's form
    // where the server serves it (server_form: strided dense, sparse and offset/length rings)
    const int tb = g_tune_pkt_bound.load();
    if (!((tb >= 0 && tb <= 3) ? netcsum::pkt_stream_supported(a, 0, tb)
                  : netcsum::pkt_stream_supported(a, 0, kBurstBound) || netcsum::pkt_stream_supported(a, 0, 2))) {
        return NET_UTIL_ERR_NONE;
    }
    uint64_t span = 0;
    if (h_off == nullptr) {
        span = (uint64_t)(n_pkt - 1u) * stride + pkt_len;
    } else {
        for (uint32_t i = 0; i < n_pkt; ++i) span = std::max<uint64_t>(span, h_off[i] + h_len[i]);
    }
    if (span > kBurstZCSpan) return NET_UTIL_ERR_NONE;
    const uint8_t* d_ring = pinned_alias(h_base, span);
    if (d_ring == nullptr) return NET_UTIL_ERR_NONE;
    *taken = true;
    NET_ERR e = ensure_burst(c);
    if (e != NET_UTIL_ERR_NONE) return e;
    const uint64_t* d_off = nullptr;
    const uint16_t* d_len = nullptr;
    if (h_off != nullptr) {                             // descriptors: staged in coherent pinned memory
        std::memcpy(c.h_burst + kBurstOff, h_off, (size_t)n_pkt * 8u);
        std::memcpy(c.h_burst + kBurstLen, h_len, (size_t)n_pkt * 2u);
        d_off = reinterpret_cast<const uint64_t*>(c.h_burst_dev + kBurstOff);
        d_len = reinterpret_cast<const uint16_t*>(c.h_burst_dev + kBurstLen);
    }
    uint32_t form = 0, spw = 0;
    const int zc = g_tune_burst_zc.load();
    if (zc == 3 && server_form(h_off, stride, pkt_len, n_pkt, &form, &spw)) {   // the resident server
        uint8_t* hr = c.h_burst + kBurstRec;
        std::memset(hr, 0xFF, (size_t)n_pkt * 8u);
        netcsum::BurstPost p{};
        p.ring = reinterpret_cast<uint64_t>(d_ring);
        p.stride = (uint32_t)stride;
        p.n = n_pkt;
        p.pkt_len = pkt_len;
        p.spw = spw;
        p.form = (form << 1) | 1u;
        p.udp_mode = udp_mode;
        server_launch_name(form, spw, true);
        e = burst_server_run(c, p, [&](uint32_t i) { return *(volatile uint8_t*)(hr + 8u * i + 7u) != 0xFFu; }, n_pkt);
        if (e != NET_UTIL_ERR_NONE) return e;
    } else if (zc >= 2) {                               // records straight into coherent memory, polled
        uint8_t* hr = c.h_burst + kBurstRec;
        std::memset(hr, 0xFF, (size_t)n_pkt * 8u);     // sentinel: a record's store byte is 0..3
        e = pkt_batch(d_ring, d_off, d_len, stride, pkt_len, n_pkt, nullptr, udp_mode, true, 0, c.stream, nullptr, 0u,
                      nullptr, reinterpret_cast<netcsum::PktTxRecord*>(c.h_burst_dev + kBurstRec), kBurstBound);
        if (e != NET_UTIL_ERR_NONE) return e;
        mark_zero_copy_launch(2);
        e = burst_poll(c, [&](uint32_t i) { return *(volatile uint8_t*)(hr + 8u * i + 7u) != 0xFFu; }, n_pkt);
        if (e != NET_UTIL_ERR_NONE) return e;
    } else {
        netcsum::PktTxRecord* d_rec = reinterpret_cast<netcsum::PktTxRecord*>(c.d_burst + kBurstDevRec);
        e = pkt_batch(d_ring, d_off, d_len, stride, pkt_len, n_pkt, nullptr, udp_mode, true, 0, c.stream, nullptr, 0u,
                      nullptr, d_rec, kBurstBound);
        if (e != NET_UTIL_ERR_NONE) return e;
        mark_zero_copy_launch(1);
        if (++c.seq == 0u) c.seq = 1u;
        const uint32_t tag = c.seq;
        *reinterpret_cast<volatile unsigned long long*>(c.h_burst + kBurstWord) = 0ull;
        NC_HIP(netcsum::launch_burst_done(reinterpret_cast<const uint8_t*>(d_rec), nullptr, n_pkt * 8u,
                                          c.h_burst_dev + kBurstRec, nullptr,
                                          reinterpret_cast<unsigned long long*>(c.h_burst_dev + kBurstWord), tag,
                                          c.stream));
        e = burst_wait(c, tag);
        if (e != NET_UTIL_ERR_NONE) return e;
    }
    uint8_t* hb = static_cast<uint8_t*>(h_base);
    const uint64_t* rec = reinterpret_cast<const uint64_t*>(c.h_burst + kBurstRec);
    std::vector<uint64_t> walk_off;
    std::vector<uint16_t> walk_len;
    std::vector<uint32_t> walk_idx;
    for (uint32_t i = 0; i < n_pkt; ++i) {
        const uint64_t r = rec[i];                      // PktTxRecord: vals | l4_off << 32 | flags << 48 | store << 56
        const uint32_t flags = (uint32_t)(r >> 48) & 0xFFu, store = (uint32_t)(r >> 56);
        const uint64_t o = h_off ? h_off[i] : (uint64_t)i * stride;
        if (flags & NETCSUM_PKT_EXT_HDR) {
            walk_off.push_back(o);
            walk_len.push_back(h_off ? h_len[i] : pkt_len);
            walk_idx.push_back(i);
            continue;
        }
        uint8_t* p = hb + o;
        const uint16_t ip = (uint16_t)r, l4 = (uint16_t)(r >> 16);
        if (store & 1u) std::memcpy(p + 10, &ip, 2);
        if (store & 2u) std::memcpy(p + ((r >> 32) & 0xFFFFu), &l4, 2);
        if (h_flags) h_flags[i] = (uint8_t)flags;
    }
    if (!walk_off.empty()) {                            // the rare long IPv6 chains: the copy path
        const uint32_t m = (uint32_t)walk_off.size();
        std::vector<uint8_t> fl(m);
        char zc_name[256];
        snprintf(zc_name, sizeof zc_name, "%s", NetUtil_MI355X_LastLaunch());
        e = pkt_host_copy(h_base, walk_off.data(), walk_len.data(), 0, 0, m, h_flags ? fl.data() : nullptr, nullptr,
                          0u, udp_mode, true, 1u);
        if (e != NET_UTIL_ERR_NONE) return e;
        char d[256];
        snprintf(d, sizeof d, "%.180s +copy path for %u EXT_HDR datagrams", zc_name, m);
        netcsum::set_last_launch(d);
        if (h_flags) {
            for (uint32_t k = 0; k < m; ++k) h_flags[walk_idx[k]] = fl[k];
        }
    }
    return NET_UTIL_ERR_NONE;
}

// Tx records returned from the device for a chunk of a host-memory Tx batch: the checksum fields
// written into the caller's host buffer (memcpy of the bytes as the device wrote them).
static void apply_field_records(uint8_t* h_base, const uint64_t* h_off, uint64_t stride, uint32_t s0, uint32_t ns,
                                const uint64_t* rec) {
    for (uint32_t i = 0; i < ns; ++i) {
        const uint64_t r = rec[i];
        const uint32_t pos = (uint32_t)(r >> 32);
        if ((pos & (netcsum::kFieldIP | netcsum::kFieldL4)) == 0u) continue;
        uint8_t* p = h_base + (h_off ? h_off[s0 + i] : (uint64_t)(s0 + i) * stride);
        const uint16_t ip = (uint16_t)r, l4 = (uint16_t)(r >> 16);
        if (pos & netcsum::kFieldIP) std::memcpy(p + 10, &ip, 2);
        if (pos & netcsum::kFieldL4) std::memcpy(p + (pos & 0xFFFFu), &l4, 2);
    }
}

// Packet batches from host memory: RxValidateIP / TxFinalizeIP / RxBurst / TxBurst over the chunks.
// Tx: the device form runs on the chunk's copy and records which checksum fields it wrote
// (fieldpos); a gather pass packs them into 8-B records, only those return D2H, and the host writes
// the fields into its own buffer once the chunk's stream has drained (before its slot is reused,
// and at the end) — 8 B per datagram over PCIe instead of the chunk's bytes.
static NET_ERR pkt_host_copy(void* h_base, const uint64_t* h_off, const uint16_t* h_len, uint64_t stride,
                             CPU_INT16U pkt_len, uint32_t n_pkt, uint8_t* h_flags, uint8_t* h_action, uint32_t rx_cfg,
                             uint32_t udp_mode, bool tx, uint32_t n_chunks) {
    HostCtx* cp = nullptr;
    NET_ERR e = host_ctx(&cp);
    if (e != NET_UTIL_ERR_NONE) return e;
    HostCtx& c = *cp;
    std::vector<HostChunk> ch;
    // n_chunks 0 = the library's choice (tools/burst_latency.c, profiles/r3x_burst_latency.jsonl): each
    // chunk adds 15-20 us per call and PCIe stays the bound, so one chunk, except Tx from 32 Ki
    // datagrams, whose host-side field write-back overlaps the later chunks' copies (262 144 frames:
    // 16 chunks 7.4 ms, one 8.4 ms)
    if (n_chunks == 0) n_chunks = tx ? std::min(16u, std::max(1u, n_pkt / 16384u)) : 1u;
    if (n_pkt / n_chunks > (1u << 28)) n_chunks = (n_pkt >> 28) + 1u;   // records: 32-bit offsets
    const uint64_t maxb = plan_chunks(h_off, h_len, stride, pkt_len, n_pkt, n_chunks, ch);
    const bool varlen = h_off != nullptr;
    const uint32_t per = ch[0].ns;
    // device slot: [bytes | offsets | lengths | flags | actions | field positions | records];
    // host slot: [offsets | lengths | records]
    const size_t o_off = al256(maxb), o_len = o_off + al256(varlen ? (size_t)per * 8u : 0u);
    const size_t o_fl = o_len + al256(varlen ? (size_t)per * 2u : 0u), o_act = o_fl + al256(per);
    const size_t o_fp = o_act + al256(per), o_rec = o_fp + al256(tx ? (size_t)per * 4u : 0u);
    const size_t h_rec = varlen ? al256((size_t)per * 8u) + al256((size_t)per * 2u) : 0u;
    e = ensure_pipe(c, o_rec + al256(tx ? (size_t)per * 8u : 0u), h_rec + (tx ? (size_t)per * 8u : 0u));
    if (e != NET_UTIL_ERR_NONE) return e;
    PipeDrainOnExit guard{c};
    uint8_t* hb = static_cast<uint8_t*>(h_base);
    auto drain = [&](size_t k) -> NET_ERR {                  // chunk k's stream has finished: apply its records
        NC_HIP(hipStreamSynchronize(c.pstream[k % 3u]));
        if (tx) {
            apply_field_records(hb, h_off, stride, ch[k].s0, ch[k].ns,
                                reinterpret_cast<const uint64_t*>(c.h_pipe[k % 3u] + h_rec));
        }
        return NET_UTIL_ERR_NONE;
    };
    for (size_t k = 0; k < ch.size(); ++k) {
        const HostChunk& q = ch[k];
        const int j = (int)(k % 3u);
        hipStream_t st = c.pstream[j];
        uint8_t* d = c.d_pipe[j];
        if (k >= 3 && (varlen || tx)) {                      // slot j's staging is free again
            e = drain(k - 3u);
            if (e != NET_UTIL_ERR_NONE) return e;
        }
        NC_HIP(hipMemcpyAsync(d, hb + q.lo, q.hi - q.lo, hipMemcpyHostToDevice, st));
        if (varlen) {
            uint64_t* h_o = reinterpret_cast<uint64_t*>(c.h_pipe[j]);
            uint16_t* h_l = reinterpret_cast<uint16_t*>(c.h_pipe[j] + al256((size_t)per * 8u));
            for (uint32_t i = 0; i < q.ns; ++i) {
                h_o[i] = h_off[q.s0 + i] - q.lo;
                h_l[i] = h_len[q.s0 + i];
            }
            NC_HIP(hipMemcpyAsync(d + o_off, h_o, (size_t)q.ns * 8u, hipMemcpyHostToDevice, st));
            NC_HIP(hipMemcpyAsync(d + o_len, h_l, (size_t)q.ns * 2u, hipMemcpyHostToDevice, st));
        }
        uint32_t* d_fp = tx ? reinterpret_cast<uint32_t*>(d + o_fp) : nullptr;
        if (tx) NC_HIP(hipMemsetAsync(d_fp, 0, (size_t)q.ns * 4u, st));   // a packet no kernel wrote: no fields
        const uint64_t* d_o = varlen ? reinterpret_cast<const uint64_t*>(d + o_off) : nullptr;
        e = pkt_batch(d, d_o, varlen ? reinterpret_cast<const uint16_t*>(d + o_len) : nullptr, stride, pkt_len, q.ns,
                      h_flags ? d + o_fl : nullptr, udp_mode, tx, 0, st, h_action ? d + o_act : nullptr, rx_cfg, d_fp);
        if (e != NET_UTIL_ERR_NONE) return e;
        if (h_flags) NC_HIP(hipMemcpyAsync(h_flags + q.s0, d + o_fl, q.ns, hipMemcpyDeviceToHost, st));
        if (h_action) NC_HIP(hipMemcpyAsync(h_action + q.s0, d + o_act, q.ns, hipMemcpyDeviceToHost, st));
        if (tx) {
            netcsum::PktBatchArgs g{};
            g.base = d;
            g.off = d_o;
            g.stride = stride;
            g.n = q.ns;
            g.fieldpos_out = d_fp;
            uint64_t* d_rec = reinterpret_cast<uint64_t*>(d + o_rec);
            NC_HIP(netcsum::launch_pkt_field_gather(g, d_rec, st));
            NC_HIP(hipMemcpyAsync(c.h_pipe[j] + h_rec, d_rec, (size_t)q.ns * 8u, hipMemcpyDeviceToHost, st));
        }
    }
    for (size_t k = ch.size() > 3 ? ch.size() - 3 : 0; k < ch.size(); ++k) {
        e = drain(k);
        if (e != NET_UTIL_ERR_NONE) return e;
    }
    guard.done = true;
    return NET_UTIL_ERR_NONE;
}

static NET_ERR pkt_host(void* h_base, const uint64_t* h_off, const uint16_t* h_len, uint64_t stride, CPU_INT16U pkt_len,
                        uint32_t n_pkt, uint8_t* h_flags, uint8_t* h_action, uint32_t rx_cfg, uint32_t udp_mode, bool tx,
                        uint32_t n_chunks) {
    if (n_pkt == 0) return NET_UTIL_ERR_NONE;
    if (n_pkt > 0x7FFFFFFFu) return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
    if (h_base == nullptr || (h_off != nullptr) != (h_len != nullptr) || (!tx && h_flags == nullptr && h_action == nullptr)) {
        return NET_ERR_FAULT_NULL_PTR;
    }
    if (n_chunks == 0 && g_tune_burst_zc.load() != 0) {   // a burst from a pinned ring: in place
        HostCtx* cp = nullptr;
        NET_ERR e = host_ctx(&cp);
        if (e != NET_UTIL_ERR_NONE) return e;
        bool taken = false;
        e = tx ? tx_burst_zero_copy(*cp, h_base, h_off, h_len, stride, pkt_len, n_pkt, h_flags, udp_mode, &taken)
               : rx_burst_zero_copy(*cp, h_base, h_off, h_len, stride, pkt_len, n_pkt, h_flags, h_action, rx_cfg, &taken);
        if (taken) return e;
    }
    return pkt_host_copy(h_base, h_off, h_len, stride, pkt_len, n_pkt, h_flags, h_action, rx_cfg, udp_mode, tx, n_chunks);
}

NET_ERR NetUtil_MI355X_RxValidateIPHost(const void* h_base, const uint64_t* h_off, const uint16_t* h_len, uint64_t stride,
                                        CPU_INT16U pkt_len, uint32_t n_pkt, uint8_t* h_flags, uint32_t n_chunks) {
    if (n_pkt != 0 && h_flags == nullptr) return NET_ERR_FAULT_NULL_PTR;
    return pkt_host(const_cast<void*>(h_base), h_off, h_len, stride, pkt_len, n_pkt, h_flags, nullptr, 0u, 1u, false,
                    n_chunks);
}

NET_ERR NetUtil_MI355X_TxFinalizeIPHost(void* h_base, const uint64_t* h_off, const uint16_t* h_len, uint64_t stride,
                                        CPU_INT16U pkt_len, uint32_t n_pkt, uint8_t* h_flags, int udp_tx_csum,
                                        uint32_t n_chunks) {
    return pkt_host(h_base, h_off, h_len, stride, pkt_len, n_pkt, h_flags, nullptr, 0u, udp_tx_csum ? 1u : 0u, true,
                    n_chunks);
}

NET_ERR NetUtil_MI355X_RxBurstHost(const void* h_base, const uint64_t* h_off, const uint16_t* h_len, uint64_t stride,
                                   CPU_INT16U pkt_len, uint32_t n_pkt, uint32_t rx_cfg, uint8_t* h_action,
                                   uint8_t* h_flags, uint32_t n_chunks) {
    if (n_pkt != 0 && h_action == nullptr) return NET_ERR_FAULT_NULL_PTR;
    if (rx_cfg & ~(uint32_t)NETCSUM_RXCFG_UDP_DISCARD_NO_CHK_SUM) return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
    return pkt_host(const_cast<void*>(h_base), h_off, h_len, stride, pkt_len, n_pkt, h_flags, h_action, rx_cfg, 1u,
                    false, n_chunks);
}

NET_ERR NetUtil_MI355X_TxBurstHost(void* h_base, const uint64_t* h_off, const uint16_t* h_len, uint64_t stride,
                                   CPU_INT16U pkt_len, uint32_t n_pkt, uint8_t* h_flags, uint32_t n_chunks) {
    return pkt_host(h_base, h_off, h_len, stride, pkt_len, n_pkt, h_flags, nullptr, 0u, 2u, true, n_chunks);
}

NET_ERR NetUtil_MI355X_Fill(void* d_buf, uint64_t n_bytes, uint64_t first_byte, uint64_t seed, int pattern,
                            void* hip_stream) {
    if (n_bytes == 0) return NET_UTIL_ERR_NONE;
    if (d_buf == nullptr) return NET_ERR_FAULT_NULL_PTR;
    if (((uintptr_t)d_buf & 7u) != 0u || pattern < 0 || pattern > 3) {
        return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
    }
    int dev = 0;
    NC_HIP(hipGetDevice(&dev));
    const uint64_t words = (n_bytes >> 3) + 1u;
    const uint64_t cap = (uint64_t)cu_count(dev) * 8u;
    const int grid = (int)std::max<uint64_t>(1u, std::min<uint64_t>((words + 255u) / 256u, cap));
    NC_HIP(netcsum::launch_fill(d_buf, n_bytes, first_byte, seed, pattern, grid, static_cast<hipStream_t>(hip_stream)));
    return NET_UTIL_ERR_NONE;
}

NET_ERR NetUtil_MI355X_ReadStream(const void* d_buf, uint64_t n_bytes, uint64_t* d_sink, void* hip_stream) {
    if (n_bytes == 0) return NET_UTIL_ERR_NONE;
    if (d_buf == nullptr || d_sink == nullptr) return NET_ERR_FAULT_NULL_PTR;
    if (((uintptr_t)d_buf & 15u) != 0u || (n_bytes & 15u) != 0u) return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
    int dev = 0;
    NC_HIP(hipGetDevice(&dev));
    if (g_tune_probe.load() >= 2) {                     // run-stream form (netcsum_stream.hip); 3: with a pause per piece
        NC_HIP(netcsum::launch_read_run(d_buf, n_bytes, reinterpret_cast<unsigned long long*>(d_sink),
                                        static_cast<hipStream_t>(hip_stream), g_tune_probe.load() == 3));
        return NET_UTIL_ERR_NONE;
    }
    int grid = g_tune_grid.load();
    if (grid <= 0) grid = cu_count(dev) * 32;
    NC_HIP(netcsum::launch_read_stream(d_buf, n_bytes / 16u, reinterpret_cast<unsigned long long*>(d_sink), grid,
                                       g_tune_nt.load() != 0, static_cast<hipStream_t>(hip_stream), g_tune_probe.load()));
    return NET_UTIL_ERR_NONE;
}

NET_ERR NetUtil_MI355X_PlanBind(uint32_t plan_id) {
    tls_plan_id = plan_id;
    return NET_UTIL_ERR_NONE;
}

NET_ERR NetUtil_MI355X_Tune(int key, int value) {
    switch (key) {
    case NETCSUM_TUNE_GRID_BLOCKS:
        if (value < 0) return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
        g_tune_grid.store(value);
        return NET_UTIL_ERR_NONE;
    case NETCSUM_TUNE_GROUP_LANES:
        if (!(value == 0 || value == 1 || value == 4 || value == 8 || value == 16 || value == 32 || value == 64)) {
            return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
        }
        g_tune_group.store(value);
        return NET_UTIL_ERR_NONE;
    case NETCSUM_TUNE_NT_LOADS:
        g_tune_nt.store(value < 0 ? -1 : (value != 0));
        return NET_UTIL_ERR_NONE;
    case NETCSUM_TUNE_KERNEL:
        if (value < 0 || value > 8) return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
        g_tune_kernel.store(value);
        return NET_UTIL_ERR_NONE;
    case NETCSUM_TUNE_CHUNKS:
        if (!(value == 0 || value == 1 || value == 2 || value == 3 || value == 4 || value == 6 || value == 8)) {
            return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
        }
        g_tune_chunks.store(value);
        return NET_UTIL_ERR_NONE;
    case NETCSUM_TUNE_GRID_MULT:
        if (value < 0 || value > 64) return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
        g_tune_grid_mult.store(value == 0 ? 1 : value);
        return NET_UTIL_ERR_NONE;
    case NETCSUM_TUNE_TILE:
        if (value < -1 || value > (1 << 20)) return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
        g_tune_tile.store(value);
        return NET_UTIL_ERR_NONE;
    case NETCSUM_TUNE_PROBE:
        if (value < 0 || value > 3) return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
        g_tune_probe.store(value);
        return NET_UTIL_ERR_NONE;
    case NETCSUM_TUNE_TX_PASSES:
        if (value < 0 || value > 2) return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
        g_tune_tx_passes.store(value);
        return NET_UTIL_ERR_NONE;
    case NETCSUM_TUNE_STREAM_WAVES:
        if (value != -1 && value != 0 && (value < 3 || value > 8)) return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
        netcsum::set_stream_waves(value);
        return NET_UTIL_ERR_NONE;
    case NETCSUM_TUNE_STREAM_XCD:
        if (value < -1 || value > 4096) return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
        netcsum::set_stream_xcd(value);
        return NET_UTIL_ERR_NONE;
    case NETCSUM_TUNE_TX_FLUSH:
        if (value < -1 || value > 4) return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
        netcsum::set_tx_flush(value);
        return NET_UTIL_ERR_NONE;
    case NETCSUM_TUNE_STREAM_TOUCH:
        if (value < -1 || value > 1) return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
        netcsum::set_stream_touch(value);
        return NET_UTIL_ERR_NONE;
    case NETCSUM_TUNE_CRC_KERNEL:
        if (value < 0 || value > 3) return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
        netcsum::set_crc_kernel(value);
        return NET_UTIL_ERR_NONE;
    case NETCSUM_TUNE_CRC_LANES:
        if (!(value == 0 || value == 1 || value == 2 || value == 4 || value == 8 || value == 16)) {
            return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
        }
        netcsum::set_crc_lanes(value);
        return NET_UTIL_ERR_NONE;
    case NETCSUM_TUNE_VARLEN_RUN_BYTES:
        if (value < -1 || value > (1 << 20)) return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
        netcsum::set_varlen_run_bytes(value);
        return NET_UTIL_ERR_NONE;
    case NETCSUM_TUNE_HDR_BURST:
        if (value < -1 || value > 1) return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
        netcsum::set_hdr_burst(value);
        return NET_UTIL_ERR_NONE;
    case NETCSUM_TUNE_CRC_WIDE:
        if (value < 0 || value > 2) return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
        netcsum::set_crc_wide(value);
        return NET_UTIL_ERR_NONE;
    case NETCSUM_TUNE_CRC_NT:
        if (value < 0 || value > 1) return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
        netcsum::set_crc_nt(value);
        return NET_UTIL_ERR_NONE;
    case NETCSUM_TUNE_BURST_ZERO_COPY:
        if (value < 0 || value > 3) return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
        g_tune_burst_zc.store(value);
        return NET_UTIL_ERR_NONE;
    case NETCSUM_TUNE_BURST_SERVER_IDLE_US:
        if (value < 1 || value > 1000000) return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
        g_tune_burst_idle.store(value);
        return NET_UTIL_ERR_NONE;
    case NETCSUM_TUNE_BURST_SERVER_LIFE_US:
        if (value < 1 || value > 1000000) return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
        g_tune_burst_life.store(value);
        return NET_UTIL_ERR_NONE;
    case NETCSUM_TUNE_STORE_GATHER:
        if (value < -1 || value > 1) return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
        netcsum::set_store_gather(value);
        return NET_UTIL_ERR_NONE;
    case NETCSUM_TUNE_CHAIN_GRID:
        if (value < -1 || value > 16) return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
        netcsum::set_chain_grid(value);
        return NET_UTIL_ERR_NONE;
    case NETCSUM_TUNE_CHAIN_COMBINE:
        if (value != -1 && value != 16 && value != 64) return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
        g_tune_chain_combine.store(value);
        return NET_UTIL_ERR_NONE;
    case NETCSUM_TUNE_LIVE_COMPACT:
        if (value < -1 || value > 1) return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
        netcsum::set_live_compact(value);
        return NET_UTIL_ERR_NONE;
    case NETCSUM_TUNE_PLAN_AHEAD:
        if (value < -1 || value > 1) return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
        g_tune_plan_ahead.store(value);
        return NET_UTIL_ERR_NONE;
    case NETCSUM_TUNE_FAULT_INJECT:
        if (value < 0 || value > 1) return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
        netcsum::set_fault_skip_deferred(value == 1);
        return NET_UTIL_ERR_NONE;
    case NETCSUM_TUNE_PKT_BOUND:
        if (value < -1 || value > 4) return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
        g_tune_pkt_bound.store(value);
        return NET_UTIL_ERR_NONE;
    case NETCSUM_TUNE_BLOCK_THREADS:
        if (value != 0 && value != 64 && value != 128 && value != 256) {   // __launch_bounds__(256)
            return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
        }
        g_tune_block.store(value == 0 ? 256 : value);
        return NET_UTIL_ERR_NONE;
    default:
        return (NET_ERR)NET_UTIL_ERR_MI355X_INVALID_ARG;
    }
}

const char* NetUtil_MI355X_LastLaunch(void) {
    return netcsum::last_launch();
}

const char* NetUtil_MI355X_Version(void) {
    return "netcsum-mi355x 0.1.0 gfx950";
}

}  // extern "C"
