// netcsum_hdrstream.hip — gfx950 run-stream kernel for PACKED dword-aligned short segments
// (config C3: 16 M x 20-B IPv4 headers back to back; NetUtil_16BitOnesCplChkSumHdrCalc / HdrVerify,
// net_util.c:159-195 / :245-284, whose sum is NetUtil_16BitSumHdrCalc, net_util.c:1160-1208).
//
// A wave owns a run of consecutive headers and reads their bytes as 1-KiB pieces straight into
// registers (lane l: bytes [16l, 16l + 16) of the piece, every wave-instruction 8 whole aligned
// lines, no LDS round trip, no idle lanes). With M = len / 4 dwords per header (M = 4 or 5:
// 16- or 20-B headers) every header boundary is a dword boundary and a lane's four dwords hold the
// tail of at most one header and the head of at most one other:
//   A_l = the lane's dwords before its first header start (b_l), B_l = the rest (b_l = 4: none).
// A header starting in lane l-1 (at b_{l-1}) ends in lane l-1 or lane l, so its exact half-word sum
// is B_{l-1} + A_l — one DPP wave_shr per piece (lane 0 takes lane 63's B of the previous piece
// from a scalar carry). Lane l then finishes that header (fold, complement / compare) and all lanes
// store their results with ONE store instruction (51 of 64 lanes for 20-B headers). Header
// indices and starts are pure index arithmetic, per lane, no shuffles.
//
// Arithmetic: base and length are multiples of 4, so every header starts at an even address
// (v_sad_u16 little-endian half-word sums need no rotation) and ~fold16 is the reference's
// host-order return value (netcsum_kernels.hip header).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>

#include "netcsum_device.h"
#include "netcsum_kernels.h"
#include "netcsum_stream.h"

namespace netcsum {

namespace {

using namespace sv;

// DPP wave_shr:1 (gfx9 family): lane l gets lane l-1's value, lane 0 gets `old`.
__device__ __forceinline__ uint32_t wave_shr1(uint32_t old, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x138, 0xF, 0xF, false);
}

// BURST: a whole run's results (spw <= kBurstMax) are gathered in LDS and written by one store
// instruction of whole 16-B pieces (the run's 2 spw or spw result bytes are 16-B aligned and
// contiguous), instead of one 2-B (1-B) store instruction per piece; a short last run stores per piece.
constexpr uint32_t kBurstMax = 384u;

template <int M, int D, bool NT, bool BURST>
__global__ void __launch_bounds__(256) seg_hdrstream_kernel(SegBatchArgs A, uint32_t spw) {
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t blk = A.xcd ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
    const uint64_t sb64 = ((uint64_t)blk * 4u + w) * spw;
    if (sb64 >= A.n_seg) {
        return;
    }
    const uint32_t s_begin = (uint32_t)sb64;
    const uint32_t nres = min(A.n_seg - s_begin, spw);
    const uintptr_t a_first = (uintptr_t)A.base + (uint64_t)s_begin * (4u * M);
    const uintptr_t O = a_first & ~(uintptr_t)127;
    const int r0 = (int)((a_first - O) >> 2);                 // run-relative dword of header 0
    const int rend = r0 + M * (int)nres;                       // one past the run's last dword
    const uint32_t span = 4u * (uint32_t)rend;
    const uint32_t npieces = (span + 1023u) >> 10;
    const __amdgpu_buffer_rsrc_t rd = run_rsrc(O, (span + 15u) & ~15u);   // whole 16-B loads; bytes past
                                                                           // rend are masked below
    const bool verify = A.verify != 0u;
    // The output V# must be provably wave-uniform: built from plain arithmetic the compiler kept it
    // in VGPRs and wrapped every store in a readfirstlane "waterfall" loop; readfirstlane on its
    // parts puts it in SGPRs (one store instruction per piece).
    const uint64_t ob = (uint64_t)(uintptr_t)A.out + (uint64_t)s_begin * (verify ? 1u : 2u);
    const uint32_t ob_lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)ob);
    const uint32_t ob_hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(ob >> 32));
    const __amdgpu_buffer_rsrc_t ro = run_rsrc((uintptr_t)(((uint64_t)ob_hi << 32) | ob_lo),
                                               (uint32_t)__builtin_amdgcn_readfirstlane((int)(nres * (verify ? 1u : 2u))));
    const uint32_t lane16 = 16u * lane;
    __shared__ __attribute__((aligned(16))) uint32_t res[BURST ? 4 : 1][BURST ? kBurstMax / 2 : 1];   // 768 B per wave
    const bool burst = BURST && nres == spw && spw <= kBurstMax && (spw & 15u) == 0u;   // wave-uniform

    u32x4 dv[D];
#pragma unroll
    for (int j = 0; j < D; ++j) {
        dv[j] = buf_load16<NT>(rd, ((uint32_t)j << 10) + lane16);
    }
    const RunTouch touch = touch_run(rd, npieces, lane, A.touch != 0u);    // row touch (netcsum_stream.h)

    // First header start at or after run-relative dword r (r may be below r0), as an offset from r.
    auto first_start = [&](int r) -> int {
        if (r <= r0) return r0 - r;
        const int t = (r - r0) % M;
        return t ? M - t : 0;
    };

    uint32_t carry = 0u;                                       // B of lane 63 of the previous piece
    auto consume = [&](uint32_t q, u32x4 v) {
        const int rl = 256 * (int)q + 4 * (int)lane;           // this lane's dword 0
        uint32_t s[4] = {v.x, v.y, v.z, v.w};
        uint32_t p[5];
        p[0] = 0u;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int r = rl + i;
            const uint32_t si = (r >= r0 && r < rend) ? __builtin_amdgcn_sad_u16(s[i], 0u, 0u) : 0u;
            p[i + 1] = p[i] + si;
        }
        const int b = first_start(rl);                         // this lane's first header start
        const bool has = b < 4 && rl + b < rend;
        const uint32_t Al = has ? (b == 0 ? 0u : b == 1 ? p[1] : b == 2 ? p[2] : p[3]) : p[4];
        const uint32_t Bl = p[4] - Al;
        // the previous lane (lane 63 of the previous piece for lane 0): its header start, if any
        const int rp = rl - 4;
        const int bp = first_start(rp);
        const bool hp = bp < 4 && rp + bp < rend && rp + bp >= r0;
        const uint32_t Bp = wave_shr1(carry, Bl);
        carry = (uint32_t)__builtin_amdgcn_readlane((int)Bl, 63);
        const uint32_t k = hp ? (uint32_t)((rp + bp - r0) / M) : 0u;   // run-relative header index
        const uint32_t t = fold16(Bp + Al);
        if (burst) {
            if (hp) {
                if (verify) {
                    reinterpret_cast<uint8_t*>(res[w])[k] = (uint8_t)(t == 0xFFFFu ? 1u : 0u);
                } else {
                    reinterpret_cast<uint16_t*>(res[w])[k] = (uint16_t)(~t);
                }
            }
        } else if (verify) {
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(t == 0xFFFFu ? 1u : 0u), ro, (int)(hp ? k : kOOB), 0, 0);
        } else {
            __builtin_amdgcn_raw_buffer_store_b16((uint16_t)(~t), ro, (int)(hp ? 2u * k : kOOB), 0, 0);
        }
    };

    // A header is finished by the lane after the one it starts in: only when the run's last header
    // starts in lane 63 of the last piece does that lane lie one piece past the run (zeros).
    const int rs = rend - M;
    const uint32_t total = npieces + ((((rs >> 2) & 63) == 63 && (uint32_t)(rs >> 8) == npieces - 1u) ? 1u : 0u);
    const uint32_t rounds = (total + (uint32_t)D - 1u) / (uint32_t)D;
    for (uint32_t r = 0; r < rounds; ++r) {
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const uint32_t q = r * (uint32_t)D + (uint32_t)j;
            consume(q, opaque_tuple(dv[j]));                   // pieces past `total`: zeros, no stores
            // Refills past the run read zeros without memory traffic. Branching around them (or peeling
            // the last round) was measured: the uniform branch makes the compiler drain vmcnt(0) at
            // every piece, the peeled round was 2-3 % slower (profiles/r2c3p_*).
            dv[j] = buf_load16<NT>(rd, ((q + (uint32_t)D) << 10) + lane16);   // past the run: zeros
            asm volatile("" ::: "memory");
        }
    }
    if (burst) {                       // the wave's LDS writes retire in order before its reads
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const uint32_t nbytes = verify ? spw : 2u * spw;
        if (lane16 < nbytes) {
            const u32x4 v = *reinterpret_cast<const u32x4*>(reinterpret_cast<const uint8_t*>(res[w]) + lane16);
            __builtin_amdgcn_raw_buffer_store_b128(v, ro, (int)lane16, 0, 0);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    touch_retire(touch);
}

thread_local TuneKnob g_hdr_burst{-1};      // NETCSUM_TUNE_HDR_BURST: -1 default (kHdrBurstDefault), 0, 1
constexpr bool kHdrBurstDefault = true;     // C3 0.0584 -> 0.0571-0.0575 ms (profiles/r2zi_c3_burst_sweep.jsonl)

}  // namespace

void set_hdr_burst(int v) { g_hdr_burst.store(v); }
bool hdr_burst() { const int v = g_hdr_burst.load(); return v < 0 ? kHdrBurstDefault : v > 0; }

namespace {

template <int M, int D, bool NT>
hipError_t launch_hs_t(const SegBatchArgs& a0, uint32_t spw, hipStream_t s) {
    SegBatchArgs a = a0;
    a.touch = stream_touch(true) ? 1u : 0u;
    a.xcd = stream_xcd(false) ? 1u : 0u;   // r2x: 0.0579-0.0584 ms off vs 0.0589 on
    const uint64_t waves = ((uint64_t)a.n_seg + spw - 1u) / spw;
    const dim3 grid((unsigned)((waves + 3u) / 4u));
    if (hdr_burst()) {
        hipLaunchKernelGGL((seg_hdrstream_kernel<M, D, NT, true>), grid, dim3(256), stream_lds_bytes(0), s, a, spw);
    } else {
        hipLaunchKernelGGL((seg_hdrstream_kernel<M, D, NT, false>), grid, dim3(256), stream_lds_bytes(0), s, a, spw);
    }
    return hipGetLastError();
}

}  // namespace


// Packed (stride == len), no pseudo-header, len 16 or 20, base a multiple of 4; runs < 2^31 bytes.
bool hdrstream_supported(const SegBatchArgs& a) {
    return a.seg_off == nullptr && a.pseudo == nullptr && (a.seg_len == 16u || a.seg_len == 20u) &&
           a.seg_stride == a.seg_len && ((uintptr_t)a.base & 3u) == 0u && a.n_seg < 0x7FFFFFFFu;
}

hipError_t launch_hdrstream(const SegBatchArgs& a, int depth, uint32_t spw, bool nt, hipStream_t s) {
    if (!hdrstream_supported(a) || spw == 0u || spw > (1u << 20)) return hipErrorInvalidValue;
    const int m = (int)(a.seg_len / 4u);
#define NETCSUM_HS(M_, D_, NT_) \
    if (m == M_ && depth == D_ && nt == NT_) return launch_hs_t<M_, D_, NT_>(a, spw, s);
    NETCSUM_HS(5, 4, true) NETCSUM_HS(5, 4, false) NETCSUM_HS(5, 8, true) NETCSUM_HS(5, 8, false)
    NETCSUM_HS(4, 4, true) NETCSUM_HS(4, 4, false) NETCSUM_HS(4, 8, true) NETCSUM_HS(4, 8, false)
#undef NETCSUM_HS
    return hipErrorInvalidValue;
}

}  // namespace netcsum
