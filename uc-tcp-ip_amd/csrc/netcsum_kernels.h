// netcsum_kernels.h — internal interface between the C ABI (netcsum_abi.hip) and the kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace netcsum {

// A launch option (NetUtil_MI355X_Tune): one value per calling host thread, so one thread's tuning
// never changes another thread's launches; a new thread starts from the defaults.
struct TuneKnob {
    int v;
    template <class... A>
    int load(A...) const { return v; }
    void store(int x) { v = x; }
};

struct SegBatchArgs {
    const uint8_t*  base;          // strided: first segment; varlen: base of the offsets
    const uint64_t* seg_off;       // varlen only (nullptr => strided)
    const uint16_t* seg_len_v;     // varlen only
    uint64_t        seg_stride;    // strided only
    uint32_t        seg_len;       // strided only
    const uint8_t*  pseudo;        // nullptr => no pseudo-header
    uint32_t        pseudo_stride;
    uint32_t        pseudo_len;
    uint32_t        n_seg;
    uint32_t        verify;        // 0: u16 checksum out, 1: u8 DEF_OK/DEF_FAIL out
    uint32_t        tile;          // 0: grid-stride; J > 0: block b owns segments [b*gpb*J, (b+1)*gpb*J)
    void*           out;
    uint32_t        touch;         // run-stream kernels: row-touch prologue (set by the launcher)
    uint32_t        xcd;           // stream kernels: XCD-aware block order (set by the launcher)
    const uint32_t* run_dev;       // varlen stream kernel: run length chosen on the device (used when
                                   // larger than the launch's), nullptr = the launch's
    uint32_t*       plan_out;      // varlen live kernel: the batch's plan for the next batch on the same
    uint32_t        plan_tag;      // descriptors (an extra sampler block), nullptr = none
    uint32_t        gather;        // dense stream kernel: a block's results gathered in LDS and stored as
                                   // one line by its last wave (set by the launcher)
    const uint32_t* n_dev;         // chain pass 1 (live kernel, CH): the segment count on the device
                                   // (chain_first[n]); n_seg is then the records' capacity
};

struct LaunchCfg {
    int  grid;             // workgroups; <= 0: fill the chip exactly (resident blocks x CUs x grid_mult)
    int  grid_mult;        // residency multiple used when grid <= 0
    int  cus;              // compute units of the device
    uint64_t blocks_needed;  // upper bound: one group per segment
    int  block;            // threads per workgroup (multiple of 64)
    int  group_lanes;      // lanes per segment: 1, 4, 8, 16, 32, 64
    int  chunks_per_pass;  // 16-B chunks per lane per pass: 1..4
    bool nt;               // non-temporal segment loads
    int  kernel;           // 1: seg_batch_kernel (one segment in flight per group), 2: seg_pipe_kernel,
                           // 3: seg_lds_kernel, 4: seg_tile_kernel (strided only),
                           // 5: seg_small_kernel (small 4-B-aligned strided segments, no pseudo),
                           // 6: seg_stream_kernel (dense strided runs, one wave per run),
                           // 7: seg_hdr_kernel (small headers through LDS-image tiles)
                           // 8: seg_hdrstream_kernel (packed 16 / 20-B headers, one wave per run)
    int  tile;             // segments per group per block in tile mode (0 = grid-stride)
    int  tile_pieces;      // v4: KiB of LDS image per stage (P)
    uint32_t stream_spw;   // kernel 6: segments per wave (one contiguous run each)
    uint32_t run_bytes;    // kernel 6, varlen: runs of about this many bytes, sized on the device from
                           // sampled lengths (stream_spw is then the shortest run the grid allows)
};

struct PktBatchArgs {
    const uint8_t*  base;          // packet i starts at base + off[i] (varlen) or base + i*stride
    const uint64_t* off;           // nullptr => strided
    const uint16_t* len;           // varlen: bytes of packet i present in the buffer
    uint64_t        stride;
    uint32_t        len_u;         // strided: bytes present per packet
    uint32_t        n;
    uint8_t*        flags_out;     // NETCSUM_PKT_* per packet (optional for Tx)
    uint32_t        tile;          // segments (packets) per group per block tile (0 = grid-stride)
    uint32_t        udp_tx_csum;   // Tx UDP checksums: 1 = compute, 0 = transmit none (write 0), 2 = per
                                   // datagram: a field of 0 is left 0 (no checksum), any other computed
    uint32_t        touch;         // run-stream form: row-touch prologue (set by the launcher)
    uint8_t*        action_out;    // Rx: NETCSUM_RX_* action per packet (optional; rx_action)
    uint32_t        rx_cfg;        // Rx: NETCSUM_RXCFG_* bits for the actions
    uint32_t*       defer_word;    // IPv6 / mixed: set to defer_tag by a batch kernel that leaves a
    uint32_t        defer_tag;     // datagram EXT_HDR; the walk pass runs only when it holds the tag
    uint32_t        xcd;           // run-stream form: XCD-aware block order (set by the launcher)
    uint32_t*       fieldpos_out;  // Tx (optional): per packet, which checksum fields were written —
                                   // kFieldIP | kFieldL4 | transport field offset (host-memory forms)
    uint32_t        plan;          // run-stream strided form, the next batch's plan (pkt_plan_block):
                                   // bits 0-7 the whole-span run (0: form 0 not allowed, gaps > 64 B),
                                   // bits 8-15 the longest live-piece run allowed (the bitmap's reach,
                                   // the batch size), bits 16-30 the host's tag for the ring
    uint32_t*       plan_out;      // optional: an extra block samples the batch and stores 1 << 31 |
                                   // tag << 16 | run << 8 | waves << 4 | form here (coherent host
                                   // memory); offset/length batches: bits 0-7 of `plan` unused
    uint32_t        res_waves;     // launcher: waves per SIMD to keep resident (3..8; 0: as many as fit)
    uint32_t*       vl_list;       // offset/length runs not in address order within the reach: the
    uint32_t*       vl_ctr;        // stream kernel appends their indices (vl_ctr[0]: count, by atomic
                                   // add) and the deferred pass (pkt_vl_deferred_kernel) does them, then
                                   // leaves vl_ctr[0..1] zero; nullptr: done inline
    uint32_t        vl_wide;       // launcher: the deferred pass's grid, wide (1) or 8 blocks (0)
};
constexpr uint32_t kFieldIP = 1u << 31;    // fieldpos_out: the IPv4 header checksum field (+10) written
constexpr uint32_t kFieldL4 = 1u << 30;    // fieldpos_out: the transport field at (bits 0-15) written
// One 8-B record per packet of a host-memory Tx batch (pkt_field_gather_kernel): the written field
// values as they lie in memory (IP | transport << 16), the transport offset << 32, and the
// kFieldIP / kFieldL4 bits << 32 (bits 62 / 63).
hipError_t launch_pkt_field_gather(const PktBatchArgs& a, uint64_t* rec_out, hipStream_t s);

// Tx UDP checksum policy of a datagram whose checksum field holds `field` (PktBatchArgs::udp_tx_csum).
__host__ __device__ __forceinline__ bool udp_tx_compute(uint32_t mode, uint32_t field) {
    return mode == 1u || (mode == 2u && field != 0u);
}

// Two-pass Tx (run-stream form): one record per packet between the checksum pass and the scatter pass,
// written and read as ONE little-endian uint64 (vals | l4_off << 32 | flags << 48 | store << 56).
struct PktTxRecord {
    uint32_t vals;         // IP checksum | transport checksum << 16 (host order)
    uint16_t l4_off;       // packet offset of the transport checksum field
    uint8_t  flags;        // NETCSUM_PKT_* verdict
    uint8_t  store;        // bit 0: write the IP field, bit 1: write the transport field
};

struct ChainBatchArgs {
    const uint8_t*  base;          // piece j starts at base + off[j]
    const uint64_t* off;
    const uint16_t* len;
    const uint32_t* first;         // chain i = pieces [first[i], first[i+1])
    const uint8_t*  pseudo;        // nullptr => no pseudo-header
    uint32_t        pseudo_stride;
    uint32_t        pseudo_len;
    uint32_t        n;
    uint32_t        verify;
    void*           out;
    uint32_t        xcd;           // pass 1: XCD-aware tile order (set by the launcher)
};

hipError_t launch_chain_batch(const ChainBatchArgs& a, int group, int grid, hipStream_t s);
// Two-pass form (default): per-piece even/odd sums into `eo` (cap records), then a combine pass per
// chain; batches of more than `cap` pieces fall back to the wave-per-chain form inside pass 2.
// live_spw != 0: pass 1 in the live-sector stream, runs of live_spw (<= 64) consecutive pieces,
// live_depth (4 / 8) pieces in flight.
// NETCSUM_TUNE_CHAIN_GRID: 0 / -1 pass 1 in tiles of 64 pieces, one per block; k >= 1 a grid of k x the
// resident blocks, each owning an equal contiguous share of the pieces
void set_chain_grid(int v);
int chain_grid();
hipError_t launch_chain_two_pass(const ChainBatchArgs& a, uint64_t* eo, uint32_t cap, int cus, hipStream_t s,
                                 uint32_t live_spw = 0u, int live_depth = 8);
// Chain pass 1 in the live-sector segment stream (seg_live_varlen_kernel<…, CH>, netcsum_stream.hip):
// runs of spw (<= 64) consecutive pieces, depth (4 / 8) pieces in flight, compacted sectors when cmp;
// each piece's exact half-word sum (u32, absolute LE frame) into rec[j]. Then the combine pass over
// those records (chain_combine_h_kernel, netcsum_chains.hip); the two together:
hipError_t launch_chain_live_records(const ChainBatchArgs& c, uint32_t* rec, uint32_t cap, int depth, uint32_t spw, bool cmp,
                                     hipStream_t s);
// combine_lanes: 16 or 64 lanes per chain in the combine pass
hipError_t launch_chain_two_pass_h(const ChainBatchArgs& a, uint32_t* rec, uint32_t cap, int cus, hipStream_t s,
                                   uint32_t spw, int depth, bool cmp, int combine_lanes);

// CRC-32 batches (netcsum_crc.hip; net_util.c:485-636).
struct CrcBatchArgs {
    const uint8_t*  base;          // segment i at base + off[i] (varlen) or base + i * stride
    const uint64_t* off;           // nullptr => strided
    const uint32_t* lens;          // varlen lengths (nullptr => all `len`)
    uint64_t        stride;
    uint32_t        len;
    uint32_t        n;
    uint32_t        cpl;           // 0: NetUtil_32BitCRC_Calc, 1: NetUtil_32BitCRC_CalcCpl
    uint32_t*       out;
    uint32_t        xs[4];         // strided: x^(8 s 2^k) mod P of the 16-lane combine (set by the launcher)
    uint32_t        xl;            // strided: x^(8 len) mod P
};
constexpr uint32_t kCrcShortMax = 96u;     // strided segments up to this length: one lane each
hipError_t launch_crc_batch(const CrcBatchArgs& a, uint32_t max_len, int cus, hipStream_t s);
const char* crc_launch_name(uint32_t max_len, bool varlen);
void set_crc_kernel(int v);    // NETCSUM_TUNE_CRC_KERNEL
void set_crc_nt(int v);        // NETCSUM_TUNE_CRC_NT
void set_crc_lanes(int v);     // NETCSUM_TUNE_CRC_LANES
void set_crc_wide(int v);      // NETCSUM_TUNE_CRC_WIDE

hipError_t launch_pkt_batch(const PktBatchArgs& a, const LaunchCfg& c, bool tx, int ip_ver,  // 4, 6, 0 = per packet
                            hipStream_t s);

bool tile_supported(int g, int p, int k);   // is (G, P, K) a compiled v4 instantiation
const char* last_launch();                  // description of this thread's last batch launch

hipError_t launch_seg_batch(const SegBatchArgs& a, const LaunchCfg& c, hipStream_t s);
bool small_supported(const SegBatchArgs& a);  // strided, no pseudo, 1..64 B, base/stride 4-B aligned
hipError_t launch_small_batch(const SegBatchArgs& a, int grid, hipStream_t s);
bool hdr_supported(const SegBatchArgs& a);     // small_supported and stride <= 64: LDS-image header tiles
int hdr_lanes_h(const SegBatchArgs& a, int h);  // headers per lane kernel 7 uses for a request (auto: h <= 0)
uint32_t hdr_pieces(const SegBatchArgs& a, int h);   // 1-KiB LDS-DMA pieces per tile of 64*h headers
int hdr_occupancy(const SegBatchArgs& a, int stages, int h);
bool hdrstream_supported(const SegBatchArgs& a);                  // kernel 8: packed 16 / 20-B headers
hipError_t launch_hdrstream(const SegBatchArgs& a, int depth, uint32_t spw, bool nt, hipStream_t s);
// Varlen run length from sampled lengths: *out = clamp(run_bytes / (mean length + extra), spw_min, 128);
// with plan_out, also the batch's plan there: 1 << 31 | tag << 16 | form (0 the stream kernel; 1 / 2
// the lane-group pipe at 16 x 6 / 8 x 8, for sparse pools; 3 the live-sector stream, run << 8, bit 2
// depth 8).
hipError_t launch_varlen_runlen(const uint64_t* offs, const uint16_t* lens, uint32_t n, uint32_t extra, uint32_t run_bytes,
                                uint32_t spw_min, uint32_t* out, uint32_t* plan_out, uint32_t tag, hipStream_t s);
// Segments one per pool buffer (plan 3): the live-sector stream (netcsum_stream.hip
// seg_live_varlen_kernel), runs of spw <= 64 segments, depth 4 or 8 pieces in flight; a.plan_out:
// one extra block samples the descriptors for the next batch's plan.
hipError_t launch_live_varlen(const SegBatchArgs& a, int depth, uint32_t spw, hipStream_t s);
void set_varlen_run_bytes(int v);   // NETCSUM_TUNE_VARLEN_RUN_BYTES
// NETCSUM_TUNE_LIVE_COMPACT: the live-sector streams read their live sectors compacted, 16 per
// wave-instruction (-1 default / 1), or as the live 1-KiB pieces of their span (0)
void set_live_compact(int v);
bool live_compact();
// NETCSUM_TUNE_STORE_GATHER: the dense segment stream kernel's results, per block of 4 runs, gathered in
// LDS and stored whole by the block's last wave (-1 default / 1), or per wave (0)
void set_store_gather(int v);
bool store_gather();
uint32_t varlen_run_bytes();
constexpr uint32_t kVarlenSpwMin = 3u;
void set_hdr_burst(int v);     // NETCSUM_TUNE_HDR_BURST: header stream results written per run (1) or per piece (0)
bool hdr_burst();
bool pkt_stream_supported(const PktBatchArgs& a, int ip_ver, int bound);   // run-stream packet kernel's domain
// Tx finalize write-back of the dirty field lines (NETCSUM_TUNE_TX_FLUSH): -1 / 0 none, 1 scatter
// stores at system scope, 2 release at the end of every scatter wave, 3 / 4 a write-back launch of
// 8 / 256 workgroups after the Tx launch(es).
void set_tx_flush(int mode);
// bound (NETCSUM_TUNE_PKT_BOUND): 0 every piece of the run's span, 1 / 2 / 3 the live pieces, with 0 / 1
// / depth pieces loaded during the parse (netcsum_pktstream.hip; depth 8: bounds 0, 2 and 3)
// rec: two-pass Tx (records + scatter); scatter = false: the records only (zero-copy host bursts, whose
// host applies them)
hipError_t launch_pkt_stream(const PktBatchArgs& a, int ip_ver, int depth, uint32_t spw, bool nt, bool tx, int bound,
                             hipStream_t s, PktTxRecord* rec = nullptr, bool scatter = true);
// The ring plan's sampler alone (one block; a.plan, a.plan_out and the batch's descriptors / stride as
// for the batch): the plan word for the batch about to be launched, which the host waits for.
hipError_t launch_pkt_plan(const PktBatchArgs& a, int ip_ver, hipStream_t s);
// Test-only fault (NETCSUM_TUNE_FAULT_INJECT 1): the calling thread's next offset/length packet batch
// with a deferred pass enqueues its stream kernel, skips the deferred pass and fails with
// hipErrorLaunchFailure — the state a failed deferred launch leaves (the list counters not reset).
void set_fault_skip_deferred(bool on);
// Zero-copy host bursts: one wave copies n result bytes (flags, and actions if act != nullptr) from
// device memory into coherent pinned host memory, then stores `tag` into *word (system scope).
hipError_t launch_burst_done(const uint8_t* fl, const uint8_t* act, uint32_t n, uint8_t* h_fl, uint8_t* h_act,
                             unsigned long long* word, uint32_t tag, hipStream_t s);

// Resident burst server (NETCSUM_TUNE_BURST_ZERO_COPY 3; netcsum_pktstream.hip burst_server_kernel):
// the host posts a zero-copy burst as ONE 64-B line of coherent host memory, which the server's
// leader waves poll, instead of launching a kernel per burst.
// Live-piece runs (run-stream packet kernels, bounds 1-3) span at most 63 KiB from their first 128-B
// line: piece 63 is never live, and its bit is the pop's sentinel.
constexpr uint32_t kLiveReach = 63u << 10;

struct alignas(64) BurstPost {
    uint64_t seq;          // burst number, increasing; kBurstStop: exit
    uint64_t ring;         // device address of the ring (its pinned alias)
    uint32_t stride;       // strided forms
    uint32_t n;            // frames (<= 4096)
    uint32_t pkt_len;      // strided forms: bytes present per slot
    uint32_t spw;          // frames per wave run
    uint32_t form;         // bit 0 Tx; form >> 1: kBurstWhole / kBurstLive / kBurstOffLen
    uint32_t udp_mode;     // Tx: PktBatchArgs::udp_tx_csum
    uint32_t rx_cfg;       // Rx: NETCSUM_RXCFG_* for the actions
    uint32_t check;        // burst_post_check of the fields above: a read that tore the line fails it
    uint32_t pad[4];
};
static_assert(sizeof(BurstPost) == 64, "one line");
constexpr uint64_t kBurstStop = ~0ull;
constexpr uint32_t kBurstWhole = 0u, kBurstLive = 1u, kBurstOffLen = 2u;
constexpr int kBurstServerMaxBlocks = 16;
__host__ __device__ __forceinline__ uint32_t burst_post_check(const BurstPost& p) {
    const uint32_t d[11] = {(uint32_t)p.seq, (uint32_t)(p.seq >> 32), (uint32_t)p.ring, (uint32_t)(p.ring >> 32),
                            p.stride, p.n, p.pkt_len, p.spw, p.form, p.udp_mode, p.rx_cfg};
    uint32_t h = 0x811C9DC5u;                               // FNV-1a over the dwords
    for (int i = 0; i < 11; ++i) h = (h ^ d[i]) * 0x01000193u;
    return h;
}
struct BurstServerArgs {
    const BurstPost*    post;      // device alias of the post line
    unsigned long long* closed;    // [blocks]: set by a block that stops serving (device-written)
    uint8_t*            flags;     // Rx results (device aliases of coherent host memory)
    uint8_t*            act;
    PktTxRecord*        rec;       // Tx records
    const uint64_t*     off;       // offset/length descriptors (staged in coherent host memory)
    const uint16_t*     len;
    uint64_t            seq0;      // the last burst number already served
    uint64_t            idle_ticks;   // wall-clock ticks without a post after which a block stops
    uint64_t            life_ticks;   // wall-clock ticks after the block's start after which it stops
                                      // even while bursts keep coming (bounds how long the server holds
                                      // the hardware queue its stream shares with other streams)
};
// blocks x 256 threads on stream s (a stream of its own: the kernel runs until it is idle)
hipError_t launch_burst_server(const BurstServerArgs& a, int blocks, hipStream_t s);
// IPv6 extension-header chains past the batch kernels' window (flags EXT_HDR): walked to the end and
// finished in place (netcsum_v6walk.hip); a.flags_out holds the batch kernel's flags.
hipError_t launch_pkt_v6_walk(const PktBatchArgs& a, bool tx, int cus, hipStream_t s);
void set_last_launch(const char* desc);
hipError_t launch_hdr_batch(const SegBatchArgs& a, int stages, int h, int grid, hipStream_t s);
bool stream_supported(const SegBatchArgs& a);  // strided, stride in [len, len+64], len >= 256
bool stream_dense(const SegBatchArgs& a);      // strided, stride == len >= 1024: the default for kernel 6
uint32_t stream_spw(const SegBatchArgs& a, uint64_t waves);
int stream_occupancy(int depth, const SegBatchArgs& a, bool nt);   // resident 256-thread blocks per CU
hipError_t launch_stream_batch(const SegBatchArgs& a, int depth, uint32_t spw, bool nt, hipStream_t s);
// Residency cap of the run-stream kernels (NETCSUM_TUNE_STREAM_WAVES, -1 = each kernel's default):
// LDS bytes each 256-thread workgroup reserves so that at most w of them (w waves per SIMD) fit a
// CU's 160 KiB; 0 = no cap.
void set_stream_waves(int w);
uint32_t stream_lds_bytes(int auto_waves);
bool stream_waves_tuned();             // NETCSUM_TUNE_STREAM_WAVES set (>= 0)
// Row-touch prologue of the run-stream kernels (NETCSUM_TUNE_STREAM_TOUCH: -1 each kernel's
// default `auto_on`, 0 off, 1 on).
void set_stream_touch(int t);
bool stream_touch(bool auto_on);
// XCD-aware block order of the segment / varlen / header stream kernels (NETCSUM_TUNE_STREAM_XCD:
// -1 each kernel's default `auto_on`, 0 off, 1 on). Measured (profiles/r2w_*, r2x_*): C5 shard
// 3.614 -> 3.561 ms, C2 0.2186 -> 0.2181, C4 0.6777 -> 0.6747 (on); C3 0.0579-0.0584 -> 0.0589 (off).
void set_stream_xcd(int on);
bool stream_xcd(bool auto_on);
// the block-order mode for xcd_block (netcsum_stream.h): 0 dispatch order, 1 one slice per XCD, C >= 2
// chunks of C blocks per XCD in turn; auto_mode when the knob is at its default (-1)
uint32_t stream_xcd_mode(uint32_t auto_mode);
hipError_t launch_stream_exact(const void* d_p, uint32_t n16, unsigned long long* d_sum, int grid,
                               hipStream_t s, uint32_t tag = 0u);   // tag != 0 (grid 1): completion word
hipError_t launch_fill(void* d_buf, uint64_t n_bytes, uint64_t first_byte, uint64_t seed, int pattern, int grid,
                       hipStream_t s);
hipError_t launch_read_stream(const void* d_p, uint64_t n16, unsigned long long* d_sink, int grid, bool nt,
                              hipStream_t s, int variant);
hipError_t launch_read_run(const void* d_p, uint64_t n_bytes, unsigned long long* d_sink, hipStream_t s, bool sleep);

}  // namespace netcsum
