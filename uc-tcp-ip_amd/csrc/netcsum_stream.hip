// netcsum_stream.hip — gfx950 "segmented stream" kernel for dense strided segment batches
// (configs C2 / C5: 1500 B TCP segments + 12 B IPv4 pseudo-headers, one
// NetUtil_16BitOnesCplChkSumDataCalc / ...DataVerify per segment, net_util.c:344-363, :428-449;
// the sum itself is NetUtil_16BitSumDataCalc, net_util.c:1321-1475, plus the pseudo-header partial
// of NetUtil_16BitOnesCplSumDataCalc, net_util.c:1591-1609).
//
// Why a third form. The lane-group kernels (netcsum_kernels.hip) give every segment its own G
// lanes, so a wave-instruction reads G-lane pieces at 16-B alignment and the 16-B chunks that
// straddle two segments are fetched twice. Here a WAVE owns a contiguous run of segments and reads
// their bytes exactly like a pure read stream: piece q of the wave is the 1 KiB at O + 1024*q
// (O = 128-B line below the first segment), lane l holds its 16 B at O + 1024*q + 16*l — every
// wave-instruction is 8 whole, aligned cache lines and every byte of the run is fetched once.
// Segment boundaries are wave-uniform scalar events: while consuming piece q the wave walks (on
// the SALU) the segments that END inside it; for each, every lane takes the bytes of that segment
// in its chunk (a VALU prefix mask), the 64 shares are reduced with four DPP row shifts and four
// v_readlane, and the scalar epilogue (fold, parity rotation, + the pseudo-header sum, complement)
// leaves the result in lane k % 64 of two VGPRs, stored with one coalesced store per run.
//
// Pseudo-headers (12 B for IPv4 TCP/UDP, net_tcp.h:1545-1551) are summed in a per-run prologue
// (lane k = segment k, 16-B-aligned chunks, all loads issued together) while the run's first
// pieces are in flight.
//
// Loads are raw buffer loads (V# over the wave's byte run, voffset = 1024*q + 16*lane): the
// hardware range check returns zeros past the run, so the pipeline's dummy pieces and unused pseudo
// lanes need no zero-chunk address select. D pieces are in flight per wave (register ring,
// counted vmcnt, `opaque` keeps every stage's wait in straight-line code — netcsum_device.h).
//
// Arithmetic (bit-exact; see netcsum_kernels.hip): absolute 16-B frame, v_sad_u16 little-endian
// half-word sums, per-lane exact partials (< 2^26 for a 64 KiB segment), per-lane fold16 + the
// segment's parity rotation, DPP sum of 64 folded values (< 2^23), fold16, complement.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <atomic>

#include "netcsum_device.h"
#include "netcsum_kernels.h"
#include "netcsum_stream.h"

namespace netcsum {

namespace {

using namespace sv;

constexpr uint32_t kMaxRun = 128u;     // segments per wave run: results live in two VGPRs (lane = k % 64)
constexpr uint64_t kMaxGap = 64u;      // varlen runs stream across gaps of up to this many bytes

// Pseudo-header sums of run segments [s_begin, s_begin + nres): lane k % 64 of ps0 (k < 64) / ps1
// holds segment k's pseudo-header sum, folded, in its own stream frame, from the 16-B-aligned chunks
// that cover it (all loads issued before any is used). PH 1: <= 2 chunks per header, 2: <= 5.
template <int PH>
struct PseudoChunks {
    static constexpr int kPch = PH == 1 ? 2 : 5;              // chunks one pseudo-header can touch
    u32x4 v[2][kPch];
};

template <int PH>
__device__ __forceinline__ void run_pseudo_issue(const SegBatchArgs& A, uint32_t s_begin, uint32_t nres, uint32_t lane,
                                                 PseudoChunks<PH>& P) {
    const uint32_t plen = A.pseudo_len;
    const uint32_t pst = A.pseudo_stride;
    const uintptr_t pfirst = (uintptr_t)A.pseudo + (uint64_t)s_begin * pst;
    const uintptr_t PB = pfirst & ~(uintptr_t)15;
    const uint32_t plead = (uint32_t)(pfirst - PB);
    const uint32_t pspan = plead + (nres - 1u) * pst + plen;
    const __amdgpu_buffer_rsrc_t rp = run_rsrc(PB, (pspan + 15u) & ~15u);
    const uint32_t nchmax = (plen + 30u) >> 4;                 // chunks one pseudo-header can touch
    constexpr int kPch = PseudoChunks<PH>::kPch;
    auto& pv = P.v;
#pragma unroll
    for (int sl = 0; sl < 2; ++sl) {
        const uint32_t k = lane + 64u * (uint32_t)sl;
        const uint32_t a = plead + k * pst;
        const uint32_t hi = (a & 15u) + plen;
#pragma unroll
        for (int i = 0; i < kPch; ++i) {
            // PH 1 (<= 17 B: both chunks, a chunk past the header at kOOB): no branch, so that no load is
            // pending on one path only — the waitcnt pass would drain vmcnt(0) at the join, i.e. wait
            // for the run's first pieces here (run_pseudo_issue's loads are consumed after the stream)
            if (PH == 1 || (uint32_t)i < nchmax) {             // wave-uniform
                const uint32_t off = (k < nres && 16u * (uint32_t)i < hi) ? (a & ~15u) + 16u * (uint32_t)i : kOOB;
                pv[sl][i] = buf_load16<false>(rp, off);
            } else {
                pv[sl][i] = u32x4{0u, 0u, 0u, 0u};
            }
        }
    }
}

template <int PH>
__device__ __forceinline__ void run_pseudo_finish(const SegBatchArgs& A, uint32_t s_begin, uint32_t lane,
                                                  const PseudoChunks<PH>& P, uint32_t& ps0, uint32_t& ps1) {
    const uint32_t plen = A.pseudo_len;
    const uint32_t pst = A.pseudo_stride;
    const uint32_t plead = (uint32_t)(((uintptr_t)A.pseudo + (uint64_t)s_begin * pst) & 15u);
    constexpr int kPch = PseudoChunks<PH>::kPch;
    const auto& pv = P.v;
#pragma unroll
    for (int sl = 0; sl < 2; ++sl) {
        const uint32_t k = lane + 64u * (uint32_t)sl;
        const uint32_t a = plead + k * pst;
        const int lo = (int)(a & 15u);
        const int hi = lo + (int)plen;
        uint32_t acc = 0u;
#pragma unroll
        for (int i = 0; i < kPch; ++i) {
            const int b = 16 * i;
            acc += low_bytes(pv[sl][i], min(max(hi - b, 0), 16)) - low_bytes(pv[sl][i], min(max(lo - b, 0), 16));
        }
        uint32_t s = fold16(acc);
        if (a & 1u) {
            s = rot8(s);
        }
        if (sl == 0) {
            ps0 = s;
        } else {
            ps1 = s;
        }
    }
}

template <int PH>
__device__ __forceinline__ void run_pseudo_sums(const SegBatchArgs& A, uint32_t s_begin, uint32_t nres, uint32_t lane,
                                                uint32_t& ps0, uint32_t& ps1) {
    PseudoChunks<PH> P;
    run_pseudo_issue<PH>(A, s_begin, nres, lane, P);
    run_pseudo_finish<PH>(A, s_begin, lane, P, ps0, ps1);
}

// Scalar epilogue shared by the stream kernels: the folded result of run segment k from the wave
// total T of its bytes (absolute LE frame; `odd`: the segment starts at an odd stream position),
// plus its pseudo-header sum, complemented (Calc) or compared (Verify), into lane k % 64 of r0/r1.
template <int PH>
__device__ __forceinline__ void finish_segment(uint32_t k, uint32_t T, bool odd, bool verify, uint32_t lane,
                                               uint32_t ps0, uint32_t ps1, uint32_t& r0, uint32_t& r1) {
    uint32_t t = fold16(T);
    if (odd) {
        t = rot8(t);
    }
    if constexpr (PH != 0) {
        const uint32_t p0 = (uint32_t)__builtin_amdgcn_readlane((int)ps0, (int)(k & 63u));
        const uint32_t p1 = (uint32_t)__builtin_amdgcn_readlane((int)ps1, (int)(k & 63u));
        t = fold16(t + (k < 64u ? p0 : p1));
    }
    const uint32_t val = verify ? (t == 0xFFFFu ? 1u : 0u) : (~t & 0xFFFFu);
    r0 = (lane == k) ? val : r0;
    r1 = (lane + 64u == k) ? val : r1;
}

__device__ __forceinline__ void store_run_results(const SegBatchArgs& A, uint32_t s_begin, uint32_t nres,
                                                  uint32_t lane, uint32_t r0, uint32_t r1) {
    if (A.verify) {
        uint8_t* o = static_cast<uint8_t*>(A.out) + s_begin;
        if (lane < nres) o[lane] = (uint8_t)r0;
        if (lane + 64u < nres) o[lane + 64u] = (uint8_t)r1;
    } else {
        uint16_t* o = static_cast<uint16_t*>(A.out) + s_begin;
        if (lane < nres) o[lane] = (uint16_t)r0;
        if (lane + 64u < nres) o[lane + 64u] = (uint16_t)r1;
    }
}

// One wave = segments [s_begin, s_end) of a strided batch (stride >= len >= 1, run <= 128 segments).
// ONE: stride == len >= 1024, so at most one segment ends inside any 1-KiB piece and the next one
// starts at that same byte — the per-piece work is one uniform branch, and an event is one prefix
// mask, one DPP reduction and a scalar epilogue. Otherwise the general walk (any number of events
// per piece, gaps between segments).
// PH: 0 no pseudo-header, 1 pseudo-headers touching <= 2 aligned chunks (<= 17 B), 2 up to 64 B.
// Results of a block's 4 consecutive runs (4 x 16 segments in C2 / C5: 128 B of u16 checksums, one
// aligned line) gathered in LDS and stored by the wave that finishes last, instead of 32 B per wave:
// on some boxes the C5 shard ran at 84 % of spec against 90 % on others while its read probe did not
// move (profiles/r6e_*: the kernel's L2 tag stalls 3.7 x those of a fast box, its translations no
// different), i.e. the partial-line result stores, whose lines leave the L2 before their neighbours'
// stores arrive once the stream exceeds what the caches hold.
constexpr uint32_t kGatherMax = 4u * kMaxRun;

__device__ __forceinline__ void gather_store_results(const SegBatchArgs& A, uint32_t blk, uint32_t w, uint32_t spw,
                                                     uint32_t nres, uint32_t lane, uint32_t r0, uint32_t r1,
                                                     uint16_t* res, uint32_t* cnt) {
    const uint32_t k0 = w * spw;                               // this wave's results within the block
    if (lane < nres) res[k0 + lane] = (uint16_t)r0;
    if (lane + 64u < nres) res[k0 + lane + 64u] = (uint16_t)r1;
    const uint64_t b0 = (uint64_t)blk * 4u * spw;              // the block's first segment
    const uint64_t left = (uint64_t)A.n_seg - b0;
    const uint32_t nw = (uint32_t)min<uint64_t>(4u, (left + spw - 1u) / spw);   // waves of the block with a run
    uint32_t old = 0u;
    if (lane == 0u) {
        old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    old = (uint32_t)__builtin_amdgcn_readfirstlane((int)old);
    if (old + 1u == nw) {                                      // the last: the block's results, whole lines
        const uint32_t tot = (uint32_t)min<uint64_t>(4u * spw, left);
        if (A.verify) {
            uint8_t* o = static_cast<uint8_t*>(A.out) + b0;
            for (uint32_t i = lane; i < tot; i += 64u) o[i] = (uint8_t)res[i];
        } else {
            uint16_t* o = static_cast<uint16_t*>(A.out) + b0;
            for (uint32_t i = lane; i < tot; i += 64u) o[i] = res[i];
        }
    }
}

template <int D, int PH, bool NT, bool ONE>
__global__ void __launch_bounds__(256) seg_stream_kernel(SegBatchArgs A, uint32_t spw) {
    __shared__ uint16_t g_res[kGatherMax];
    __shared__ uint32_t g_cnt;
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t blk = A.xcd ? xcd_block(blockIdx.x, gridDim.x, A.xcd) : blockIdx.x;
    if (A.gather) {                                            // (every wave, before any returns)
        if (threadIdx.x == 0u) g_cnt = 0u;
        __syncthreads();
    }
    const uint64_t sb64 = ((uint64_t)blk * 4u + w) * spw;
    if (sb64 >= A.n_seg) {
        return;
    }
    const uint32_t s_begin = (uint32_t)sb64;
    const uint32_t nres = min(A.n_seg - s_begin, spw);
    const uint32_t s_end = s_begin + nres;

    const uint32_t L = A.seg_len;
    const uint32_t st = (uint32_t)A.seg_stride;
    const uintptr_t a_first = (uintptr_t)A.base + (uint64_t)s_begin * A.seg_stride;
    const uintptr_t O = a_first & ~(uintptr_t)127;
    const uint32_t span = (uint32_t)(a_first - O) + (nres - 1u) * st + L;
    const uint32_t npieces = (span + 1023u) >> 10;
    const __amdgpu_buffer_rsrc_t rd = run_rsrc(O, (span + 15u) & ~15u);
    const uint32_t lane16 = 16u * lane;
    const bool ph_odd = PH != 0 && (A.pseudo_len & 1u) != 0u;

    u32x4 dv[D];
#pragma unroll
    for (int j = 0; j < D; ++j) {                              // first D pieces in flight ...
        dv[j] = buf_load16<NT>(rd, ((uint32_t)j << 10) + lane16);
    }
    const RunTouch touch = touch_run(rd, npieces, lane, A.touch != 0u);    // row touch (netcsum_stream.h)

    // ... and the run's pseudo-headers behind them. 12-B headers (PH 1, C2 / C5): only LOADED here and
    // added in a vector epilogue after the stream, so no wave waits for them before its first piece
    // (loads return in order: they have arrived by the time the first refill is consumed) and a segment
    // end costs no pseudo-header readlanes; longer ones (PH 2, 40-B IPv6) are summed here.
    constexpr bool kDeferPseudo = PH == 1;
    uint32_t ps0 = 0u, ps1 = 0u;
    PseudoChunks<kDeferPseudo ? 1 : 2> pvd;
    if constexpr (kDeferPseudo) {
        run_pseudo_issue<1>(A, s_begin, nres, lane, pvd);
    } else if constexpr (PH != 0) {
        run_pseudo_sums<PH>(A, s_begin, nres, lane, ps0, ps1);
        touch_retire(touch);                                   // issued before the pseudo loads: retired
    }

    uint32_t res0 = 0u, res1 = 0u;                             // result of run segment k: lane k % 64
    auto finish = [&](uint32_t cur, uint32_t T, bool odd) {
        if constexpr (kDeferPseudo) {                          // the folded, rotated sum; the epilogue the rest
            uint32_t t = fold16(T);
            t = odd ? rot8(t) : t;
            const uint32_t k = cur - s_begin;
            res0 = (lane == k) ? t : res0;
            res1 = (lane + 64u == k) ? t : res1;
        } else {
            finish_segment<PH>(cur - s_begin, T, odd, A.verify != 0u, lane, ps0, ps1, res0, res1);
        }
    };

    uint32_t cur = s_begin;                                    // next segment to finish
    uint32_t cs = (uint32_t)(a_first - O);                     // its start / end, run-relative
    uint32_t ce = cs + L;
    uint32_t acc = 0u;                                         // this lane's share so far (mod 2^32)
    if constexpr (ONE) {
        const u32x4 v0 = opaque_tuple(dv[0]);                  // bytes of piece 0 before the run
        acc = 0u - piece_prefix(v0, sum4(v0, 0u), lane16, cs);
    }

    // State lives in locals inside consume and is written back unconditionally at the end: a branch
    // that updates `ce` on one side and `acc` on the other must not be merged by the optimiser into
    // one store through a phi of two addresses (that pins the state in scratch memory).
    auto consume = [&](uint32_t q, u32x4 v) {
        const uint32_t qb = q << 10;
        const uint32_t pend = qb + 1024u;
        const uint32_t full = sum4(v, 0u);
        uint32_t u = cur, c = cs, e = ce, a = acc;
        if constexpr (ONE) {
            if (u < s_end && e <= pend) {                      // segment `u` ends in this piece
                const uint32_t Pe = piece_prefix(v, full, lane16, e - qb);
                finish(u, wave_total(a + Pe), (((e - L) & 1u) != 0u) != ph_odd);
                a = full - Pe;                                 // the next segment starts at e
                ++u;
                e += st;
            } else {
                a += full;
            }
        } else {
            if (!(u < s_end && e <= pend)) {                   // no segment ends in this piece
                if (u < s_end) {
                    a += (c <= qb) ? full : full - piece_prefix(v, full, lane16, min(c - qb, 1024u));
                }
            } else {
                uint32_t Ps = (c <= qb) ? 0u : piece_prefix(v, full, lane16, c - qb);
#pragma clang loop vectorize(disable) unroll(disable)
                do {
                    const uint32_t Pe = piece_prefix(v, full, lane16, e - qb);
                    finish(u, wave_total(a + (Pe - Ps)), ((c & 1u) != 0u) != ph_odd);
                    a = 0u;
                    ++u;
                    c += st;
                    e += st;
                    Ps = (st == L) ? Pe : piece_prefix(v, full, lane16, min(c - qb, 1024u));
                } while (u < s_end && e <= pend);
                if (u < s_end) {
                    a = full - Ps;
                }
            }
        }
        cur = u;
        cs = c;
        ce = e;
        acc = a;
    };

    const uint32_t rounds = (npieces + (uint32_t)D - 1u) / (uint32_t)D;
    for (uint32_t r = 0; r < rounds; ++r) {
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const uint32_t q = r * (uint32_t)D + (uint32_t)j;
            consume(q, opaque_tuple(dv[j]));
            dv[j] = buf_load16<NT>(rd, ((q + (uint32_t)D) << 10) + lane16);   // past the run: zeros
            asm volatile("" ::: "memory");                     // keep the refill here, not sunk to the latch
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");          // trailing dummy pieces
    if constexpr (PH == 0 || kDeferPseudo) {
        touch_retire(touch);
    }
    if constexpr (kDeferPseudo) {                              // + the pseudo-header, complement / compare
        run_pseudo_finish<1>(A, s_begin, lane, pvd, ps0, ps1);
        const uint32_t t0 = fold16(res0 + ps0), t1 = fold16(res1 + ps1);
        res0 = A.verify ? (t0 == 0xFFFFu ? 1u : 0u) : (~t0 & 0xFFFFu);
        res1 = A.verify ? (t1 == 0xFFFFu ? 1u : 0u) : (~t1 & 0xFFFFu);
    }

    if (A.gather) {
        gather_store_results(A, blk, w, spw, nres, lane, res0, res1, g_res, &g_cnt);
    } else {
        store_run_results(A, s_begin, nres, lane, res0, res1);
    }
}

// Variable-length batches (offset/length descriptors, config C4). A wave takes a run of segments;
// when they are PACKED (each starts where the previous one ends — the layout of back-to-back
// datagrams) the run is one byte stream and the wave reads it exactly like seg_stream_kernel, with
// the segment bounds taken from the run's descriptors (held in VGPRs: lane k % 64 of slot k / 64) by
// v_readlane; gaps of up to kMaxGap bytes between segments are read and skipped. Any other run
// (larger gaps, reordering, overlap, a span >= 2^31) is summed four segments at a time by 16-lane
// groups — always correct; the packed layout is the fast path. (Segments in pool buffers with larger
// gaps: the batch's plan may take the lane-group pipe form instead, launch_batch.)
template <int D, int PH, bool NT>
__global__ void __launch_bounds__(256) seg_stream_varlen_kernel(SegBatchArgs A, uint32_t spw) {
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    // Adaptive runs: the grid was sized for runs of `spw`; a longer device-chosen run leaves the
    // blocks past the ones it needs idle, and the XCD order is taken over the blocks in use.
    uint32_t nwg = gridDim.x;
    if (A.run_dev != nullptr) {
        spw = max(spw, min((uint32_t)__builtin_amdgcn_readfirstlane((int)*A.run_dev), kMaxRun));
        nwg = (uint32_t)((((uint64_t)A.n_seg + spw - 1u) / spw + 3u) / 4u);
        if (blockIdx.x >= nwg) {
            return;
        }
    }
    const uint32_t blk = A.xcd ? xcd_block(blockIdx.x, nwg, A.xcd) : blockIdx.x;
    const uint64_t sb64 = ((uint64_t)blk * 4u + w) * spw;
    if (sb64 >= A.n_seg) {
        return;
    }
    const uint32_t s_begin = (uint32_t)sb64;
    const uint32_t nres = min(A.n_seg - s_begin, spw);
    const uint32_t s_end = s_begin + nres;
    const uint32_t lane16 = 16u * lane;
    const bool ph_odd = PH != 0 && (A.pseudo_len & 1u) != 0u;
    const uintptr_t base = (uintptr_t)A.base;

    // The run's descriptors: slot 0 = segments lane, slot 1 = segments 64 + lane.
    const bool v0 = lane < nres, v1 = lane + 64u < nres;
    const uint64_t off0 = v0 ? A.seg_off[s_begin + lane] : 0ull;
    const uint64_t off1 = v1 ? A.seg_off[s_begin + 64u + lane] : 0ull;
    const uint32_t len0 = v0 ? A.seg_len_v[s_begin + lane] : 0u;
    const uint32_t len1 = v1 ? A.seg_len_v[s_begin + 64u + lane] : 0u;

    uint32_t ps0 = 0u, ps1 = 0u;
    if constexpr (PH != 0) {
        run_pseudo_sums<PH>(A, s_begin, nres, lane, ps0, ps1);
    }
    uint32_t res0 = 0u, res1 = 0u;

    // Packed? Segment k starts where k - 1 ends, and the run spans < 2^31 bytes.
    const uint64_t end0 = off0 + len0, end1 = off1 + len1;
    const uint64_t prev0 = __shfl_up(end0, 1, 64);
    const uint64_t prev1_up = __shfl_up(end1, 1, 64);
    const uint64_t last0 = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(end0 >> 32), 63) << 32) |
                           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)end0, 63);
    const uint64_t prev1 = lane == 0u ? last0 : prev1_up;
    const bool ok0 = !v0 || lane == 0u || (off0 >= prev0 && off0 - prev0 <= kMaxGap);
    const bool ok1 = !v1 || (off1 >= prev1 && off1 - prev1 <= kMaxGap);
    const uint64_t first = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(off0 >> 32), 0) << 32) |
                           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)off0, 0);
    const uint32_t kl = nres - 1u;                             // last segment of the run
    const uint64_t eA = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(end0 >> 32), (int)(kl & 63u)) << 32) |
                        (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)end0, (int)(kl & 63u));
    const uint64_t eB = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(end1 >> 32), (int)(kl & 63u)) << 32) |
                        (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)end1, (int)(kl & 63u));
    const uint64_t run_end = kl < 64u ? eA : eB;
    const bool packed = __all(ok0 && ok1) && run_end >= first && run_end - first < (1ull << 31) - 256u;

    if (!packed) {
        // Scattered run: four segments at a time, a 16-lane group each (the lane-group form of
        // seg_pipe_kernel: 4 chunks per lane in flight per pass), group totals to the scalar epilogue.
        const uint32_t g = lane >> 4;
        for (uint32_t k0 = 0; k0 < nres; k0 += 4u) {          // wave-uniform loop
            const uint32_t k = k0 + g;
            const int src = (int)(k & 63u);
            const uint64_t o0 = __shfl(off0, src, 64), o1 = __shfl(off1, src, 64);
            const uint32_t l0 = (uint32_t)__shfl((int)len0, src, 64), l1 = (uint32_t)__shfl((int)len1, src, 64);
            const uintptr_t a = base + (k < 64u ? o0 : o1);
            const uint32_t len = k < nres ? (k < 64u ? l0 : l1) : 0u;
            const uint32_t tot = group_sum<16>(span_partial<16, 4, NT>(a, len, (int)(lane & 15u)));
            const uint32_t odd = (uint32_t)(((a & 1u) != 0u) != ph_odd);
#pragma unroll
            for (uint32_t i = 0; i < 4u; ++i) {
                if (k0 + i < nres) {
                    const uint32_t T = (uint32_t)__builtin_amdgcn_readlane((int)tot, (int)(16u * i));
                    const bool o = __builtin_amdgcn_readlane((int)odd, (int)(16u * i)) != 0;
                    finish_segment<PH>(k0 + i, T, o, A.verify != 0u, lane, ps0, ps1, res0, res1);
                }
            }
        }
        store_run_results(A, s_begin, nres, lane, res0, res1);
        return;
    }

    const uintptr_t a_first = base + first;
    const uintptr_t O = a_first & ~(uintptr_t)127;
    const uint32_t lead = (uint32_t)(a_first - O);
    const uint32_t span = lead + (uint32_t)(run_end - first);
    const uint32_t npieces = max(1u, (span + 1023u) >> 10);   // >= 1: a run of empty segments still ends
    const __amdgpu_buffer_rsrc_t rd = run_rsrc(O, (span + 15u) & ~15u);
    u32x4 dv[D];
#pragma unroll
    for (int j = 0; j < D; ++j) {
        dv[j] = buf_load16<NT>(rd, ((uint32_t)j << 10) + lane16);
    }
    const RunTouch touch = touch_run(rd, npieces, lane, A.touch != 0u);
    // run-relative segment starts and ends (a packed run may have gaps of <= kMaxGap bytes)
    const uint32_t rs0 = lead + (uint32_t)(off0 - first), re0 = rs0 + len0;
    const uint32_t rs1 = lead + (uint32_t)(off1 - first), re1 = rs1 + len1;
    auto pick = [&](uint32_t x0, uint32_t x1, uint32_t k) -> uint32_t {   // lane k % 64 of slot k / 64
        const uint32_t y0 = (uint32_t)__builtin_amdgcn_readlane((int)x0, (int)(k & 63u));
        const uint32_t y1 = (uint32_t)__builtin_amdgcn_readlane((int)x1, (int)(k & 63u));
        return k < 64u ? y0 : y1;
    };

    uint32_t cur = s_begin;
    uint32_t cs = lead;
    uint32_t ce = pick(re0, re1, 0u);
    uint32_t acc = 0u;
    auto consume = [&](uint32_t q, u32x4 v) {
        const uint32_t qb = q << 10;
        const uint32_t pend = qb + 1024u;
        const uint32_t full = sum4(v, 0u);
        uint32_t u = cur, c = cs, e = ce, a = acc;
        if (!(u < s_end && e <= pend)) {
            if (u < s_end) {
                a += (c <= qb) ? full : full - piece_prefix(v, full, lane16, min(c - qb, 1024u));
            }
        } else {
            uint32_t Ps = (c <= qb) ? 0u : piece_prefix(v, full, lane16, c - qb);
#pragma clang loop vectorize(disable) unroll(disable)
            do {
                const uint32_t Pe = piece_prefix(v, full, lane16, e - qb);
                finish_segment<PH>(u - s_begin, wave_total(a + (Pe - Ps)), ((c & 1u) != 0u) != ph_odd,
                                   A.verify != 0u, lane, ps0, ps1, res0, res1);
                a = 0u;
                ++u;
                const uint32_t pe = e;
                if (u < s_end) {
                    c = pick(rs0, rs1, u - s_begin);
                    e = pick(re0, re1, u - s_begin);
                }
                Ps = (c == pe) ? Pe : piece_prefix(v, full, lane16, min(c - qb, 1024u));
            } while (u < s_end && e <= pend);
            if (u < s_end) {
                a = full - Ps;
            }
        }
        cur = u;
        cs = c;
        ce = e;
        acc = a;
    };

    const uint32_t rounds = (npieces + (uint32_t)D - 1u) / (uint32_t)D;
    for (uint32_t r = 0; r < rounds; ++r) {
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const uint32_t q = r * (uint32_t)D + (uint32_t)j;
            consume(q, opaque_tuple(dv[j]));
            dv[j] = buf_load16<NT>(rd, ((q + (uint32_t)D) << 10) + lane16);
            asm volatile("" ::: "memory");
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    touch_retire(touch);
    store_run_results(A, s_begin, nres, lane, res0, res1);
}

// The plan word from the sampled mean length, mean pitch (of the pn in-order pairs of m samples):
// segments with gaps of >= 32 B between them, mostly in order, take the live-sector stream
// (seg_live_varlen_kernel): below a 455-B mean length runs as long as the reach allows (a run's slots
// span < 61 KiB: 41 1520-B buffers, 30 2-KiB ones), 16 below a 910-B mean, longer segments runs of 8
// at depth 4 in nearly dense pools (pitch < 1800 B) and of 16 at depth 8 in sparser ones
// (tools/varlen_pool_probe.py POOL_LIVE, profiles/r5t_*, r5y_*, r5ac_*: the 20 / 556 / 1480-B mix
// 0.0975 ms in runs of 32 against 0.0953 in runs of 40 in 1520-B buffers; 1480-B segments there
// 0.2211-0.2294 ms in runs of 8 at depth 4 against 0.2280-0.2305 in 16 at depth 8, in 2-KiB buffers
// 0.2522-0.2567 against 0.2574-0.2585); pools too sparse for runs of 4 take the lane-group pipe form
// (1: 16 x 6 for >= 1 KiB segments, 2: 8 x 8).
__device__ __forceinline__ uint32_t varlen_plan_word(uint32_t mlen, uint64_t ptot, uint64_t pn, uint32_t m, uint32_t tag) {
    const uint32_t pitch = (uint32_t)(ptot / max(pn, 1ull));
    const bool gapped = pn * 2u >= (uint64_t)m && pitch >= mlen + 32u;
    uint32_t form = 0u;
    if (gapped) {
        const uint32_t cap = (kLiveReach - 2048u) / max(pitch, 1u);
        const bool shrt = mlen * 45u < 20480u, lng = mlen * 45u >= 40960u;
        const bool d8 = lng && pitch >= 1800u;                 // long segments with wide gaps
        const uint32_t run = min(shrt ? 64u : (lng && !d8) ? 8u : 16u, cap);
        form = run >= 4u ? (3u | (d8 ? 4u : 0u) | (run << 8)) : (mlen >= 1024u ? 1u : 2u);
    }
    return 0x80000000u | ((tag & 0x7FFFu) << 16) | form;
}

// Sampling by one block of NTH threads (NTH / 64 waves): the mean of up to kVarlenSamples evenly
// spaced lengths and the mean in-order pitch; thread 0 returns the sums. (4096 samples took the
// one-block kernel 18-20 µs ahead of every C4 batch — one CU's misses on 12 K scattered lines,
// profiles/r5x_c4_pmc.json, r5z_*; 1024 estimate a mean length to ≈ 2 %.)
constexpr uint32_t kVarlenSamples = 1024u;
template <int NTH>
__device__ __forceinline__ void varlen_sample(const uint64_t* offs, const uint16_t* lens, uint32_t n, uint32_t m,
                                              uint32_t (&part)[NTH / 64][3], uint32_t& tot, uint64_t& ptot, uint64_t& pn) {
    uint32_t acc = 0u, pit = 0u, npit = 0u;
    // U samples per thread at a time, every load issued before any is used (the live kernel's sampler
    // block takes one at a time: its registers count toward the whole kernel's)
    constexpr int U = NTH >= 1024 ? 4 : 1;
    for (uint32_t j0 = threadIdx.x; j0 < m; j0 += (uint32_t)U * (uint32_t)NTH) {
        uint32_t l[U];
        uint64_t a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t j = j0 + (uint32_t)u * (uint32_t)NTH;
            const uint32_t i = j < m ? (uint32_t)(((uint64_t)j * n) / m) : 0u;
            l[u] = j < m ? lens[i] : 0u;
            a[u] = offs[i];
            b[u] = (j < m && i + 1u < n) ? offs[i + 1u] : 0u;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            acc += l[u];
            if (b[u] > a[u] && b[u] - a[u] < 65536u) {          // in order and near: a pitch
                pit += (uint32_t)(b[u] - a[u]);
                npit += 1u;
            }
        }
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        acc += (uint32_t)__shfl_xor((int)acc, d, 64);
        pit += (uint32_t)__shfl_xor((int)pit, d, 64);
        npit += (uint32_t)__shfl_xor((int)npit, d, 64);
    }
    if ((threadIdx.x & 63u) == 0u) {
        part[threadIdx.x >> 6][0] = acc;
        part[threadIdx.x >> 6][1] = pit;
        part[threadIdx.x >> 6][2] = npit;
    }
    __syncthreads();
    tot = 0u;
    ptot = 0u;
    pn = 0u;
    if (threadIdx.x == 0u) {
        for (int i = 0; i < NTH / 64; ++i) {
            tot += part[i][0];
            ptot += part[i][1];
            pn += part[i][2];
        }
    }
}

// Segments one per pool buffer (DataPtr + TransportHdrIx of 1520-B or 2-KiB NET_BUFs, net_util.c:1627-1628,
// 1649; net_tcp.c:1920): in address order, with gaps between them. The packed form above reads the
// gaps (or, past kMaxGap, leaves the run to its 16-lane groups); here a wave reads only the 64-B
// sectors that hold segment bytes, as the packet kernels' live pieces do (netcsum_pktstream.hip): each
// lane marks its segment's sectors in a per-wave 1024-bit LDS bitmap (a run spans < 63 KiB from its
// first 128-B line, kLiveReach), one ballot gives the run's live 1-KiB pieces, the stream pops them in
// address order (bit 63 the never-live sentinel) and lane l loads its 16 B of piece q only when its
// sector is live. Segment ends are the same scalar events as above, each leaving the segment's total
// in its lane; a segment that ends within 48 B of its first 16-B chunk (the 20-B segment of a 40-B
// ACK) is summed from that window instead, with no sectors and no event, and one vector epilogue
// finishes every lane (an empty segment: its pseudo-header alone). Each lane's first chunk is loaded
// with the plain policy before the bitmap (the live-read floor's touch, tools/live_read_probe.hip). A
// run that is not in order or outgrows the reach takes the 16-lane groups. Run length and pieces in
// flight come from the batch's plan (varlen_plan_word above; launch_batch).
constexpr uint64_t kSentinelPiece = 1ull << 63;
constexpr uint32_t kNoEnd = ~0u;

// CH (round 6): pass 1 of a NET_BUF chain batch (netcsum_chains.hip). The segments are the chain
// pieces, their count lives on the device (A.n_dev; A.n_seg is the records' capacity, a batch with
// more pieces returns at once and the combine pass takes it whole), no pseudo-header (PH 0), and each
// piece's record is its exact half-word sum T in the absolute LE frame (u32; < 2^31 for a piece of
// < 64 KiB) — one wave total per piece end, as for a segment; the combine pass applies the chain's
// stream parity.
template <int D, int PH, bool NT, bool CMP, bool CH = false>
__global__ void __launch_bounds__(256) seg_live_varlen_kernel(SegBatchArgs A, uint32_t spw) {
    __shared__ uint32_t sect_all[4][32];
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t nwg = gridDim.x;
    uint32_t nseg = A.n_seg;
    if constexpr (CH) {
        static_assert(PH == 0, "chain pieces carry no pseudo-header");
        const uint32_t np = (uint32_t)__builtin_amdgcn_readfirstlane((int)*A.n_dev);
        if (np > A.n_seg) {                                   // no room for the records
            return;
        }
        const uint32_t need = (uint32_t)(((uint64_t)np + 4ull * spw - 1u) / (4ull * spw));
        if (blockIdx.x >= need) {                             // (the grid is sized for the capacity)
            return;
        }
        nseg = np;
        nwg = need;                                           // the XCD order over the blocks with a run
    } else if (A.plan_out != nullptr) {                       // the last block: the next batch's plan
        nwg -= 1u;
        if (blockIdx.x == nwg) {
            __shared__ uint32_t part[4][3];
            const uint32_t m = min(A.n_seg, kVarlenSamples);
            uint32_t tot = 0u;
            uint64_t ptot = 0u, pn = 0u;
            varlen_sample<256>(A.seg_off, A.seg_len_v, A.n_seg, m, part, tot, ptot, pn);
            if (threadIdx.x == 0u) {
                __hip_atomic_store(A.plan_out, varlen_plan_word(m ? tot / m : 0u, ptot, pn, m, A.plan_tag),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            return;
        }
    }
    const uint32_t blk = A.xcd ? xcd_block(blockIdx.x, nwg, A.xcd) : blockIdx.x;
    const uint64_t sb64 = ((uint64_t)blk * 4u + w) * spw;
    if (sb64 >= nseg) {
        return;
    }
    const uint32_t s_begin = (uint32_t)sb64;
    const uint32_t nres = min(nseg - s_begin, spw);          // spw <= 64: segment k in lane k
    const uint32_t lane16 = 16u * lane;
    const bool ph_odd = PH != 0 && (A.pseudo_len & 1u) != 0u;
    const uintptr_t base = (uintptr_t)A.base;
    const bool mine = lane < nres;
    // lane k's pseudo-header chunks first: their addresses need no descriptor, so they travel with
    // the descriptor loads below (one memory round trip for both, not two in a row)
    constexpr int kPch = PH == 1 ? 2 : PH == 2 ? 5 : 1;
    u32x4 pv[kPch];
    uint32_t pa_lane = 0u;
    if constexpr (PH != 0) {
        const uint32_t plen = A.pseudo_len, pst = A.pseudo_stride;
        const uintptr_t pfirst = (uintptr_t)A.pseudo + (uint64_t)s_begin * pst;
        const uintptr_t PB = pfirst & ~(uintptr_t)15;
        pa_lane = (uint32_t)(pfirst - PB) + lane * pst;
        const uint32_t pspan = (uint32_t)(pfirst - PB) + (nres - 1u) * pst + plen;
        const __amdgpu_buffer_rsrc_t rp = run_rsrc(PB, (pspan + 15u) & ~15u);
        const uint32_t nchmax = (plen + 30u) >> 4;
        const uint32_t hi = (pa_lane & 15u) + plen;
#pragma unroll
        for (int c = 0; c < kPch; ++c) {
            pv[c] = (uint32_t)c < nchmax
                        ? buf_load16<false>(rp, (mine && 16u * (uint32_t)c < hi) ? (pa_lane & ~15u) + 16u * (uint32_t)c : kOOB)
                        : u32x4{0u, 0u, 0u, 0u};
        }
    }
    const uint64_t off = A.seg_off[s_begin + (mine ? lane : 0u)];
    const uint32_t len = mine ? (uint32_t)A.seg_len_v[s_begin + lane] : 0u;
    const uint64_t off0 = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(off >> 32)) << 32) |
                          (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)off);
    const uintptr_t O = (base + off0) & ~(uintptr_t)127;
    const uint64_t rel = base + off - O;                      // >= 0 when in order
    const uint64_t end = rel + len;
    const uint32_t prev_end = (uint32_t)__shfl_up((int)(uint32_t)end, 1, 64);
    const bool ok = !mine || (rel < kLiveReach && end <= kLiveReach - 128u && (lane == 0u || (uint64_t)prev_end <= rel));
    const bool stream = __builtin_amdgcn_ballot_w64(!ok) == 0u;
    const uint32_t span = stream ? (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)end, (int)(nres - 1u)) : 0u;
    const __amdgpu_buffer_rsrc_t rd = run_rsrc(O, (span + 15u) & ~15u);
    // each lane's first 16 B (plain policy: the touch), and for a segment that ends within 48 B of its
    // first chunk's start (a 20-B segment of a 40-B ACK) the next two: such a segment is summed here
    // from its window, after the stream — no sectors, no event
    const uint32_t wl = (uint32_t)rel & ~15u;
    const bool inwin = stream && mine && len != 0u && ((uint32_t)rel & 15u) + len <= 48u;
    const u32x4 w0 = buf_load16<false>(rd, (stream && mine && len != 0u) ? wl : kOOB);
    const u32x4 w1 = buf_load16<false>(rd, inwin ? wl + 16u : kOOB);
    const u32x4 w2 = buf_load16<false>(rd, inwin ? wl + 32u : kOOB);

    uint32_t ps0 = 0u, ps1 = 0u;                              // lane k: segment k's pseudo-header sum
    if constexpr (PH != 0) {
        const int lo = (int)(pa_lane & 15u), hi = lo + (int)A.pseudo_len;
        uint32_t pacc = 0u;
#pragma unroll
        for (int c = 0; c < kPch; ++c) {
            pacc += low_bytes(pv[c], min(max(hi - 16 * c, 0), 16)) - low_bytes(pv[c], min(max(lo - 16 * c, 0), 16));
        }
        ps0 = fold16(pacc);
        if (pa_lane & 1u) {
            ps0 = rot8(ps0);
        }
    }
    uint32_t res0 = 0u, res1 = 0u;
    if (!stream) {
        // out of order, overlapping or past the reach: four segments at a time, a 16-lane group each
        const uint32_t g = lane >> 4;
        for (uint32_t k0 = 0; k0 < nres; k0 += 4u) {
            const uint32_t k = k0 + g;
            const uint64_t o = __shfl(off, (int)(k & 63u), 64);
            const uint32_t l = (uint32_t)__shfl((int)len, (int)(k & 63u), 64);
            const uintptr_t a = base + o;
            // (one chunk per lane in flight: this path is rare here, and 4 set the kernel's VGPR count,
            // 72 against 40-56 — 7 waves per SIMD against 8)
            const uint32_t tot = group_sum<16>(span_partial<16, 1, NT>(a, k < nres ? l : 0u, (int)(lane & 15u)));
            const uint32_t odd = (uint32_t)(((a & 1u) != 0u) != ph_odd);
#pragma unroll
            for (uint32_t i = 0; i < 4u; ++i) {
                if (k0 + i < nres) {
                    const uint32_t T = (uint32_t)__builtin_amdgcn_readlane((int)tot, (int)(16u * i));
                    if constexpr (CH) {
                        res0 = (lane == k0 + i) ? T : res0;
                    } else {
                        const bool od = __builtin_amdgcn_readlane((int)odd, (int)(16u * i)) != 0;
                        finish_segment<PH>(k0 + i, T, od, A.verify != 0u, lane, ps0, ps1, res0, res1);
                    }
                }
            }
        }
        asm volatile("" ::"v"(w0), "v"(w1), "v"(w2));
        if constexpr (CH) {
            if (mine) static_cast<uint32_t*>(A.out)[s_begin + lane] = res0;
        } else {
            store_run_results(A, s_begin, nres, lane, res0, res1);
        }
        return;
    }

    // the run's live sectors, then its live pieces
    uint32_t* sect = sect_all[w];
    if (lane < 32u) {
        sect[lane] = 0u;
    }
    __builtin_amdgcn_wave_barrier();
    if (mine && len != 0u && !inwin) {
        const uint32_t s0 = (uint32_t)rel >> 6, s1 = ((uint32_t)end - 1u) >> 6;
        for (uint32_t d = s0 >> 5; d <= (s1 >> 5); ++d) {
            const uint32_t lo = max(s0, d << 5) - (d << 5), hi = min(s1, (d << 5) + 31u) - (d << 5);
            atomicOr(&sect[d], (2u << hi) - (1u << lo));      // bits lo..hi (hi = 31: 2 << 31 wraps to 0)
        }
    }
    __builtin_amdgcn_wave_barrier();
    const uint32_t pm0 = reinterpret_cast<const uint16_t*>(sect)[lane];
    const bool streamed = mine && len != 0u && !inwin;
    // CMP: the run's live sectors COMPACTED, in address order, 16 per wave-instruction (lane l: the
    // 16 B at (l & 3) * 16 of live sector 16 q + l / 4): a mixed pool's run holds ≈ 13 KB in ≈ 250
    // sectors spread over ≈ 60 pieces, so the piece stream below waits for ≈ 15 rounds of D partly
    // live pieces, the compacted one for ≈ 4 rounds of whole ones. A segment's bytes then lie at
    // compacted offsets [cs_l, ce_l): sector s moves to 64 x its rank among the live sectors, so byte
    // parity and 16-B alignment are kept, segments stay in address order, and the event walk below is
    // the same with those offsets (the sector bytes outside every segment are masked as gaps are).
    uint32_t nunits = 0u;                                      // pieces (or compacted pieces) to stream
    uint32_t cs_l = 0u, ce_l = 0u;                             // CMP: lane k's compacted start / end
    uint32_t nsect = 0u;                                       // CMP: the run's live sectors
    uint64_t lm0 = 0u;
    uint16_t* lst = nullptr;
    if constexpr (CMP) {
        __shared__ uint16_t lst_all[4][1024];                  // live sector indices (run-relative)
        lst = lst_all[w];
        const uint32_t cnt = (uint32_t)__builtin_popcount(pm0);
        const uint32_t incl = wave_incl_scan(cnt, lane);
        const uint32_t excl = incl - cnt;
        nsect = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        for (uint32_t m = pm0, pos = excl; m != 0u; m &= m - 1u) {
            lst[pos++] = (uint16_t)((lane << 4) | (uint32_t)__builtin_ctz(m));
        }
        auto rank = [&](uint32_t sidx) -> uint32_t {          // live sectors below sector sidx
            const int q = (int)(sidx >> 4);
            const uint32_t ex = (uint32_t)__shfl((int)excl, q, 64);
            const uint32_t pm = (uint32_t)__shfl((int)pm0, q, 64);
            return ex + (uint32_t)__builtin_popcount(pm & ((1u << (sidx & 15u)) - 1u));
        };
        const uint32_t r0 = rank(streamed ? (uint32_t)rel >> 6 : 0u);
        const uint32_t r1 = rank(streamed ? ((uint32_t)end - 1u) >> 6 : 0u);
        cs_l = streamed ? (r0 << 6) | ((uint32_t)rel & 63u) : 0u;
        ce_l = streamed ? (r1 << 6) + (((uint32_t)end - 1u) & 63u) + 1u : 0u;
        nunits = (nsect + 15u) >> 4;
        __builtin_amdgcn_wave_barrier();                       // (the list written before any lane reads it)
    } else {
        lm0 = __builtin_amdgcn_ballot_w64(pm0 != 0u);
        nunits = (uint32_t)__builtin_popcountll(lm0);
        lm0 |= kSentinelPiece;
    }
    const uint32_t lbit = 1u << (lane >> 2);
    auto pop = [&]() -> uint32_t {
        const uint32_t q = (uint32_t)__builtin_ctzll(lm0);
        lm0 = (lm0 & (lm0 - 1u)) | kSentinelPiece;
        return q;
    };
    auto live_voff = [&](uint32_t q) -> uint32_t {
        if constexpr (CMP) {                                   // compacted piece q: sector 16 q + lane / 4
            const uint32_t i = (q << 4) + (lane >> 2);
            return i < nsect ? ((uint32_t)lst[min(i, 1023u)] << 6) + ((lane & 3u) << 4) : kOOB;
        } else {
            const uint32_t sm = (uint32_t)__builtin_amdgcn_readlane((int)pm0, (int)q);
            return (sm & lbit) ? (q << 10) + lane16 : kOOB;
        }
    };
    u32x4 dv[D];
    uint32_t qd[D];
#pragma unroll
    for (int j = 0; j < D; ++j) {
        qd[j] = CMP ? (uint32_t)j : pop();
        dv[j] = buf_load16<NT>(rd, live_voff(qd[j]));
    }
    // the in-window segments' sums now, while the first pieces are in flight (the window loads were
    // issued before them, so this waits for those alone), which frees the window's 12 VGPRs before the
    // stream: 64 VGPRs, 8 waves per SIMD
    uint32_t tot = 0u;
    asm volatile("" ::"v"(w0));
    if (inwin) {                                               // [lo, hi) of the 48-B window
        const int lo = (int)((uint32_t)rel & 15u), hi = lo + (int)len;
        tot = low_bytes(w0, min(hi, 16)) - low_bytes(w0, lo) + low_bytes(w1, min(max(hi - 16, 0), 16)) +
              low_bytes(w2, max(hi - 32, 0));
    }

    // the streamed segments, in address order (lane mask), and the next one's start / end; an event
    // leaves the segment's total in its lane (tot), the epilogue below is one vector pass
    uint64_t srest = __builtin_amdgcn_ballot_w64(streamed);
    const bool any = srest != 0u;
    uint32_t cur = any ? (uint32_t)__builtin_ctzll(srest) : 63u;
    srest &= srest - 1u;
    // the next segment's start / end in the stream's frame (run-relative bytes, or compacted offsets)
    const uint32_t xs_l = CMP ? cs_l : (uint32_t)rel;
    const uint32_t xe_l = CMP ? ce_l : (uint32_t)rel + len;
    uint32_t cs = (uint32_t)__builtin_amdgcn_readlane((int)xs_l, (int)cur);
    uint32_t ce = any ? (uint32_t)__builtin_amdgcn_readlane((int)xe_l, (int)cur) : kNoEnd;
    uint32_t acc = 0u;
    auto consume = [&](uint32_t q, u32x4 v) {
        const uint32_t qb = q << 10;
        const uint32_t pend = qb + 1024u;
        const uint32_t full = sum4(v, 0u);
        uint32_t u = cur, c = cs, e = ce, a = acc, t = tot;
        uint64_t rs = srest;
        if (e > pend) {                                        // no segment ends in this piece
            a += (c <= qb) ? full : full - piece_prefix(v, full, lane16, min(c - qb, 1024u));
        } else {
            uint32_t Ps = (c <= qb) ? 0u : piece_prefix(v, full, lane16, c - qb);
#pragma clang loop vectorize(disable) unroll(disable)
            do {
                const uint32_t Pe = piece_prefix(v, full, lane16, e <= qb ? 0u : e - qb);
                const uint32_t T = wave_total(a + (Pe - Ps));
                t = (lane == u) ? T : t;
                a = 0u;
                const bool more = rs != 0u;
                u = more ? (uint32_t)__builtin_ctzll(rs) : 63u;
                rs &= rs - 1u;
                const uint32_t pe = e;
                c = (uint32_t)__builtin_amdgcn_readlane((int)xs_l, (int)u);
                e = more ? (uint32_t)__builtin_amdgcn_readlane((int)xe_l, (int)u) : kNoEnd;
                Ps = (c == pe) ? Pe : piece_prefix(v, full, lane16, c <= qb ? 0u : min(c - qb, 1024u));
            } while (e <= pend);
            a = full - Ps;
        }
        cur = u;
        srest = rs;
        cs = c;
        ce = e;
        acc = a;
        tot = t;
    };
    const uint32_t rounds = (nunits + (uint32_t)D - 1u) / (uint32_t)D;
    for (uint32_t r = 0; r < rounds; ++r) {
#pragma unroll
        for (int j = 0; j < D; ++j) {
            consume(qd[j], opaque_tuple(dv[j]));
            qd[j] = CMP ? qd[j] + (uint32_t)D : pop();         // none left: past the list / the sentinel, no loads
            dv[j] = buf_load16<NT>(rd, live_voff(qd[j]));
            asm volatile("" ::: "memory");
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (CH) {                                        // lane k: piece k's exact sum
        if (mine) static_cast<uint32_t*>(A.out)[s_begin + lane] = tot;
        return;
    }
    // vector epilogue, lane k = segment k (an empty one: its pseudo-header alone)
    uint32_t t = fold16(tot);
    if ((((uint32_t)rel & 1u) != 0u) != ph_odd) {
        t = rot8(t);
    }
    if constexpr (PH != 0) {
        t = fold16(t + ps0);
    }
    res0 = A.verify ? (t == 0xFFFFu ? 1u : 0u) : (~t & 0xFFFFu);
    store_run_results(A, s_begin, nres, lane, res0, res1);
}

template <int D, int PH, bool NT, bool CMP>
hipError_t launch_live_varlen_t(const SegBatchArgs& a0, uint32_t spw, hipStream_t s) {
    SegBatchArgs a = a0;
    a.xcd = stream_xcd_mode(1);
    const uint64_t waves = ((uint64_t)a.n_seg + spw - 1u) / spw;
    hipLaunchKernelGGL((seg_live_varlen_kernel<D, PH, NT, CMP>), dim3((unsigned)((waves + 3u) / 4u + (a.plan_out ? 1u : 0u))),
                       dim3(256), stream_lds_bytes(0), s, a, spw);
    return hipGetLastError();
}

template <int D, int PH, bool NT>
hipError_t launch_stream_varlen_t(const SegBatchArgs& a0, uint32_t spw, hipStream_t s) {
    SegBatchArgs a = a0;
    // r2ct (C4, 1 M packed 40-9000 B): runs of 8, touch, 5 waves per SIMD: 0.680 ms against 0.696 ms
    // for runs of 16 at full residency without the touch. r2zm: the best run is a byte budget, not a
    // count (C4: 3 segments = 13.6 KB, 0.657 ms; 40-1500 B: 32 segments = 25 KB, 0.158 ms against
    // 0.273 for runs of 8), so adaptive runs (run_dev) at full residency are the default.
    a.touch = stream_touch(true) ? 1u : 0u;
    a.xcd = stream_xcd_mode(1);
    const uint64_t waves = ((uint64_t)a.n_seg + spw - 1u) / spw;
    const int grid = (int)((waves + 3u) / 4u);
    hipLaunchKernelGGL((seg_stream_varlen_kernel<D, PH, NT>), dim3(grid), dim3(256),
                       stream_lds_bytes(a.run_dev != nullptr ? 0 : 5), s, a, spw);
    return hipGetLastError();
}

// One block: the mean of up to kVarlenSamples (1024) evenly spaced lengths -> run length for about run_bytes per run.
// Also the pitch — the distance from a sampled segment's start to the next one's — for the batch's
// plan (plan_out, coherent host memory, with the host's tag): segments of >= 1 KiB on average with
// gaps of >= 32 B between them (one per pool buffer, DataPtr + TransportHdrIx) read faster in the
// lane-group pipe form (16 lanes x 6 chunks, two segments in flight per group) than in the stream
// kernel, whose runs with gaps over kMaxGap take its 16-lane groups one segment at a time and whose
// packed runs read the gaps (tools/varlen_pool_probe.py, profiles/r5h_varlen_pool_probe_*.jsonl,
// r5j_*: 1480-B segments at +84 of 2-KiB buffers 0.2512 ms against 0.2817, at +34 of 1520-B buffers
// 0.2418 against 0.2484); shorter ones with gaps the pipe form at 8 lanes x 8 chunks (plan 2: the
// 40 / 576 / 1500-B mix in 1520-B buffers 0.1374 against 0.1577 in the stream kernel, r5k_*).
__global__ void __launch_bounds__(1024) varlen_runlen_kernel(const uint64_t* offs, const uint16_t* lens, uint32_t n,
                                                             uint32_t extra, uint32_t run_bytes, uint32_t spw_min,
                                                             uint32_t* out, uint32_t* plan_out, uint32_t tag) {
    __shared__ uint32_t part[16][3];
    const uint32_t m = min(n, kVarlenSamples);
    uint32_t tot = 0u;
    uint64_t ptot = 0u, pn = 0u;
    varlen_sample<1024>(offs, lens, n, m, part, tot, ptot, pn);
    if (threadIdx.x == 0u) {
        const uint32_t mlen = m ? tot / m : 0u;
        const uint32_t mean = mlen + extra;
        *out = min(max(run_bytes / max(mean, 1u), spw_min), kMaxRun);
        if (plan_out != nullptr) {
            __hip_atomic_store(plan_out, varlen_plan_word(mlen, ptot, pn, m, tag), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

}  // namespace

namespace {
thread_local TuneKnob g_varlen_run_bytes{-1};   // NETCSUM_TUNE_VARLEN_RUN_BYTES: -1 default, 0 fixed runs of 8
constexpr uint32_t kVarlenRunBytes = 16384u;
}  // namespace

void set_varlen_run_bytes(int v) { g_varlen_run_bytes.store(v); }
uint32_t varlen_run_bytes() {
    const int v = g_varlen_run_bytes.load();
    return v < 0 ? kVarlenRunBytes : (uint32_t)v;
}

hipError_t launch_varlen_runlen(const uint64_t* offs, const uint16_t* lens, uint32_t n, uint32_t extra, uint32_t run_bytes,
                                uint32_t spw_min, uint32_t* out, uint32_t* plan_out, uint32_t tag, hipStream_t s) {
    hipLaunchKernelGGL(varlen_runlen_kernel, dim3(1), dim3(1024), 0, s, offs, lens, n, extra, run_bytes, spw_min, out,
                       plan_out, tag);
    return hipGetLastError();
}

namespace {

constexpr uint32_t kXcdChunk = 256u;   // blocks per XCD chunk (xcd_block mode) for strided batches

template <int D, int PH, bool NT, bool ONE>
hipError_t launch_stream_t(const SegBatchArgs& a0, uint32_t spw, hipStream_t s) {
    SegBatchArgs a = a0;
    a.touch = stream_touch(true) ? 1u : 0u;
    // block order: one slice of the runs per XCD, or — when a slice spans >= 1 GiB — XCD chunks of
    // 256 blocks in turn. One slice per XCD puts the 8 XCDs' streams n/8 strides apart — for C5 2^23 x
    // 375 B, a multiple of 8 MiB — and on boxes where the shard's pages land that way the streams
    // collide: C5 3.772 ms against 3.521 in chunks of 256 and a read probe of 3.458 in the dispatch
    // order, the probe itself 3.659 in the slice order (profiles/r6o_c5_probe.jsonl, r6p_c5_probe.jsonl).
    // Elsewhere chunks cost 0.2-0.4 % (C5 3.517 / 3.522 against 3.507 / 3.513; C2 0.2189 against 0.2180,
    // r6n, r6q_runs.log), and C2's 200-MB slices never collided (r6e-r6p), so they keep the slices.
    const uint64_t span = (uint64_t)a.n_seg * (a.seg_stride ? a.seg_stride : a.seg_len);
    a.xcd = stream_xcd_mode(span / 8u >= (1ull << 30) ? kXcdChunk : 1u);
    a.gather = store_gather() ? 1u : 0u;
    const uint64_t waves = ((uint64_t)a.n_seg + spw - 1u) / spw;
    const int grid = (int)((waves + 3u) / 4u);
    // dense batches default to 5 waves per SIMD with the row touch: C2 0.2188 ms against 0.2346 ms
    // without either (r2ct; 0.2268 touch only, 0.2300 cap only); the residency cap's LDS reservation
    // less the kernel's static LDS (the results' gather), so that the same number of blocks fit
    const uint32_t lds = stream_lds_bytes(ONE ? 5 : 0);
    const uint32_t kStatic = kGatherMax * 2u + 16u;
    hipLaunchKernelGGL((seg_stream_kernel<D, PH, NT, ONE>), dim3(grid), dim3(256), lds > kStatic ? lds - kStatic : lds,
                       s, a, spw);
    return hipGetLastError();
}

int stream_ph(const SegBatchArgs& a) {
    if (a.pseudo == nullptr || a.pseudo_len == 0u) return 0;
    return a.pseudo_len <= 17u ? 1 : 2;
}

bool stream_one(const SegBatchArgs& a) {
    return a.seg_stride == a.seg_len && a.seg_len >= 1024u;
}

}  // namespace

namespace {

// Read-stream probe in the run-stream form (NETCSUM_TUNE_PROBE 2): a wave reads a run of
// kProbeRun bytes (C2's 16 x 1500 B) exactly like seg_stream_kernel — pieces of 1 KiB from the 128-B
// line below the run, D = 4 in flight, nt loads, the row touch, 5 waves per SIMD — and only adds the
// bytes up: the read rate the checksum kernel's access pattern can reach, with none of its arithmetic.
constexpr uint32_t kProbeRun = 16u * 1500u;

// SLEEP (NETCSUM_TUNE_PROBE 3): s_sleep 2 (~128 clocks) after each piece's sum — the same reads
// spread over a longer time per run, as the checksum kernel's per-piece work spreads them.
template <int SLEEP>
// xcd: the block order (xcd_block's mode; NETCSUM_TUNE_STREAM_XCD, default 0 here: the dispatch order).
__global__ void __launch_bounds__(256) read_run_kernel(const uint8_t* base, uint64_t n_bytes, unsigned long long* sink,
                                                       uint32_t xcd) {
    constexpr int D = 4;
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t blk = xcd ? sv::xcd_block(blockIdx.x, gridDim.x, xcd) : blockIdx.x;
    const uint64_t start = ((uint64_t)blk * 4u + w) * kProbeRun;
    if (start >= n_bytes) {
        return;
    }
    const uintptr_t a_first = (uintptr_t)base + start;
    const uintptr_t O = a_first & ~(uintptr_t)127;
    const uint32_t span = (uint32_t)(a_first - O) + (uint32_t)min<uint64_t>(kProbeRun, n_bytes - start);
    const uint32_t npieces = (span + 1023u) >> 10;
    const __amdgpu_buffer_rsrc_t rd = run_rsrc(O, (span + 15u) & ~15u);   // lead bytes read, like the kernel
    const uint32_t lane16 = 16u * lane;
    u32x4 dv[D];
#pragma unroll
    for (int j = 0; j < D; ++j) {
        dv[j] = buf_load16<true>(rd, ((uint32_t)j << 10) + lane16);
    }
    const RunTouch touch = touch_run(rd, npieces, lane, true);
    uint32_t acc = 0u;
    const uint32_t rounds = (npieces + (uint32_t)D - 1u) / (uint32_t)D;
    for (uint32_t r = 0; r < rounds; ++r) {
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const uint32_t q = r * (uint32_t)D + (uint32_t)j;
            acc = sum4(opaque_tuple(dv[j]), acc);
            if constexpr (SLEEP != 0) {
                __builtin_amdgcn_s_sleep(SLEEP);
            }
            dv[j] = buf_load16<true>(rd, ((q + (uint32_t)D) << 10) + lane16);
            asm volatile("" ::: "memory");
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    touch_retire(touch);
    if (acc == 0x9E3779B9u) {                                   // keeps the sums live; never true in practice
        sink[0] = acc;
    }
}

thread_local TuneKnob g_live_compact{-1};   // NETCSUM_TUNE_LIVE_COMPACT
thread_local TuneKnob g_store_gather{-1};   // NETCSUM_TUNE_STORE_GATHER
thread_local TuneKnob g_stream_waves{-1};
thread_local TuneKnob g_stream_touch{-1};
thread_local TuneKnob g_stream_xcd{-1};
}

hipError_t launch_read_run(const void* d_p, uint64_t n_bytes, unsigned long long* d_sink, hipStream_t s, bool sleep) {
    const uint64_t waves = (n_bytes + kProbeRun - 1u) / kProbeRun;
    const uint32_t xcd = stream_xcd_mode(0);
    if (sleep) {
        hipLaunchKernelGGL(read_run_kernel<2>, dim3((unsigned)((waves + 3u) / 4u)), dim3(256), stream_lds_bytes(5), s,
                           static_cast<const uint8_t*>(d_p), n_bytes, d_sink, xcd);
    } else {
        hipLaunchKernelGGL(read_run_kernel<0>, dim3((unsigned)((waves + 3u) / 4u)), dim3(256), stream_lds_bytes(5), s,
                           static_cast<const uint8_t*>(d_p), n_bytes, d_sink, xcd);
    }
    return hipGetLastError();
}

void set_store_gather(int v) {
    g_store_gather.store(v);
}

bool store_gather() {
    return g_store_gather.load() != 0;
}

void set_live_compact(int v) {
    g_live_compact.store(v);
}

bool live_compact() {
    return g_live_compact.load() != 0;
}

void set_stream_waves(int w) {
    g_stream_waves.store(w);
}

bool stream_waves_tuned() {
    return g_stream_waves.load(std::memory_order_relaxed) >= 0;
}

uint32_t stream_lds_bytes(int auto_waves) {
    const int g = g_stream_waves.load(std::memory_order_relaxed);
    const int w = g >= 0 ? g : auto_waves;
    // w workgroups of 4 waves per CU = w waves per SIMD: the largest 512-B multiple of which w fit
    // the 160 KiB of LDS and w + 1 do not
    return (w >= 3 && w <= 8) ? ((163840u / (uint32_t)w) & ~511u) : 0u;
}

void set_stream_touch(int t) {
    g_stream_touch.store(t);
}

void set_stream_xcd(int on) {
    g_stream_xcd.store(on);
}

bool stream_xcd(bool auto_on) {
    const int x = g_stream_xcd.load(std::memory_order_relaxed);
    return x < 0 ? auto_on : x != 0;
}

uint32_t stream_xcd_mode(uint32_t auto_mode) {
    const int x = g_stream_xcd.load(std::memory_order_relaxed);
    return x < 0 ? auto_mode : (uint32_t)x;
}

bool stream_touch(bool auto_on) {
    const int t = g_stream_touch.load(std::memory_order_relaxed);
    return t < 0 ? auto_on : t != 0;
}

// Packed segments of >= 1 KiB (stride == len): the form the library picks by default (C2, C5).
bool stream_dense(const SegBatchArgs& a) {
    return a.seg_off == nullptr && stream_one(a) && (a.pseudo == nullptr || a.pseudo_len <= 64u);
}

namespace {

template <int D>
hipError_t launch_stream_d(const SegBatchArgs& a, uint32_t spw, bool nt, hipStream_t s) {
    const int ph = stream_ph(a);
    const bool one = stream_one(a);
#define NETCSUM_L(PH_, NT_, ONE_) \
    if (ph == PH_ && nt == NT_ && one == ONE_) return launch_stream_t<D, PH_, NT_, ONE_>(a, spw, s);
#define NETCSUM_L2(PH_) NETCSUM_L(PH_, true, true) NETCSUM_L(PH_, true, false) NETCSUM_L(PH_, false, true) \
    NETCSUM_L(PH_, false, false)
    NETCSUM_L2(0) NETCSUM_L2(1) NETCSUM_L2(2)
#undef NETCSUM_L2
#undef NETCSUM_L
    return hipErrorInvalidValue;
}

}  // namespace

// Dense strided batches only: the wave reads every byte of its run, gaps included, and walks one
// scalar event per segment, so segments must be long (>= 256 B) with little or no gap between them.
bool stream_supported(const SegBatchArgs& a) {
    if (a.seg_off != nullptr) {                       // varlen: any layout (packed runs stream)
        return a.pseudo == nullptr || a.pseudo_len == 0u || a.pseudo_len <= 64u;
    }
    if (a.seg_len < 256u || a.seg_stride < a.seg_len || a.seg_stride > a.seg_len + 64u) {
        return false;
    }
    if (a.pseudo != nullptr && a.pseudo_len != 0u && a.pseudo_len > 64u) {
        return false;
    }
    return true;
}

// Segments per wave for a given number of waves: one contiguous run per wave, <= kMaxRun segments
// (results are held in two VGPRs), run byte span < 2^31.
uint32_t stream_spw(const SegBatchArgs& a, uint64_t waves) {
    uint64_t spw = ((uint64_t)a.n_seg + waves - 1u) / (waves ? waves : 1u);
    spw = std::min<uint64_t>(spw, kMaxRun);
    return (uint32_t)(spw ? spw : 1u);
}

int stream_occupancy(int depth, const SegBatchArgs& a, bool nt) {
    int occ = 0;
    hipError_t e = hipErrorInvalidValue;
    const int ph = stream_ph(a);
    const bool one = stream_one(a);
#define NETCSUM_OCC(D_, PH_, NT_, ONE_)                                                                   \
    if (depth == D_ && ph == PH_ && nt == NT_ && one == ONE_) {                                           \
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, seg_stream_kernel<D_, PH_, NT_, ONE_>, 256, 0); \
    }
#define NETCSUM_OCC2(D_, PH_) NETCSUM_OCC(D_, PH_, true, true) NETCSUM_OCC(D_, PH_, true, false) \
    NETCSUM_OCC(D_, PH_, false, true) NETCSUM_OCC(D_, PH_, false, false)
#define NETCSUM_OCC3(D_) NETCSUM_OCC2(D_, 0) NETCSUM_OCC2(D_, 1) NETCSUM_OCC2(D_, 2)
    NETCSUM_OCC3(4) NETCSUM_OCC3(6) NETCSUM_OCC3(8)
#undef NETCSUM_OCC3
#undef NETCSUM_OCC2
#undef NETCSUM_OCC
    return (e == hipSuccess && occ > 0) ? occ : 1;
}

hipError_t launch_stream_batch(const SegBatchArgs& a, int depth, uint32_t spw, bool nt, hipStream_t s) {
    if (spw == 0u || spw > kMaxRun) return hipErrorInvalidValue;
    if (a.seg_off != nullptr) {                       // varlen: depth 4 or 8
        const int ph = stream_ph(a);
#define NETCSUM_V(D_, PH_, NT_) \
        if ((depth == 8) == (D_ == 8) && ph == PH_ && nt == NT_) return launch_stream_varlen_t<D_, PH_, NT_>(a, spw, s);
        NETCSUM_V(4, 0, true) NETCSUM_V(4, 0, false) NETCSUM_V(4, 1, true) NETCSUM_V(4, 1, false)
        NETCSUM_V(4, 2, true) NETCSUM_V(4, 2, false) NETCSUM_V(8, 0, true) NETCSUM_V(8, 0, false)
        NETCSUM_V(8, 1, true) NETCSUM_V(8, 1, false) NETCSUM_V(8, 2, true) NETCSUM_V(8, 2, false)
#undef NETCSUM_V
        return hipErrorInvalidValue;
    }
    switch (depth) {
    case 4: return launch_stream_d<4>(a, spw, nt, s);
    case 6: return launch_stream_d<6>(a, spw, nt, s);
    case 8: return launch_stream_d<8>(a, spw, nt, s);
    default: return hipErrorInvalidValue;
    }
}

hipError_t launch_live_varlen(const SegBatchArgs& a, int depth, uint32_t spw, hipStream_t s) {
    if (a.seg_off == nullptr || spw == 0u || spw > 64u) return hipErrorInvalidValue;
    // PH 2 loads 5 aligned 16-B chunks of each pseudo-header: <= 64 B from any start (stream_supported's
    // limit, checked here too so that no caller can reach the kernel with a longer one)
    if (a.pseudo != nullptr && a.pseudo_len > 64u) return hipErrorInvalidValue;
    const int ph = stream_ph(a);
    const bool cmp = live_compact();
#define NETCSUM_LV(D_, PH_) \
    if (depth == D_ && ph == PH_) return cmp ? launch_live_varlen_t<D_, PH_, true, true>(a, spw, s) \
                                             : launch_live_varlen_t<D_, PH_, true, false>(a, spw, s);
    NETCSUM_LV(4, 0) NETCSUM_LV(4, 1) NETCSUM_LV(4, 2) NETCSUM_LV(8, 0) NETCSUM_LV(8, 1) NETCSUM_LV(8, 2)
#undef NETCSUM_LV
    return hipErrorInvalidValue;
}

hipError_t launch_chain_live_records(const ChainBatchArgs& c, uint32_t* rec, uint32_t cap, int depth, uint32_t spw, bool cmp,
                                     hipStream_t s) {
    if (rec == nullptr || spw == 0u || spw > 64u || cap == 0u) return hipErrorInvalidValue;
    SegBatchArgs a{};
    a.base = c.base;
    a.seg_off = c.off;
    a.seg_len_v = c.len;
    a.n_seg = cap;                                             // capacity; the count is chain_first[n]
    a.n_dev = c.first + c.n;
    a.out = rec;
    a.xcd = stream_xcd_mode(1);
    const dim3 grid((unsigned)((((uint64_t)cap + spw - 1u) / spw + 3u) / 4u));
#define NETCSUM_LC(D_)                                                                                         \
    if (depth == D_) {                                                                                         \
        if (cmp) hipLaunchKernelGGL((seg_live_varlen_kernel<D_, 0, true, true, true>), grid, dim3(256), stream_lds_bytes(0), s, a, spw); \
        else hipLaunchKernelGGL((seg_live_varlen_kernel<D_, 0, true, false, true>), grid, dim3(256), stream_lds_bytes(0), s, a, spw); \
        return hipGetLastError();                                                                              \
    }
    NETCSUM_LC(4) NETCSUM_LC(8)
#undef NETCSUM_LC
    return hipErrorInvalidValue;
}

}  // namespace netcsum
