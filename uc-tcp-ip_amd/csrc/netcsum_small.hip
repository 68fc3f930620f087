// netcsum_small.hip — gfx950 kernel for batches of SMALL, 4-byte-aligned strided segments
// (config C3: 16 M x 20 B IPv4 headers; NetUtil_16BitOnesCplChkSumHdrCalc, net_util.c:159-195,
// whose sum is NetUtil_16BitSumHdrCalc, net_util.c:1160-1208).
//
// Why a separate form: with one lane per 20-B header, the general pipelined kernel spends most of
// its instructions on 16-B-frame bookkeeping — two chunk loads per lane whose edges need
// byte masks derived from the per-lane lead, plus the pipeline's stage selects. When every segment
// starts on a 4-byte boundary (base and stride multiples of 4) and is at most 64 B long, a lane can
// load exactly its ND = ceil(len/4) dwords (dwordx4 / dwordx2 / dword at 4-B-aligned addresses,
// unaligned-access mode), mask at most the last dword, and add them with v_sad_u16: the
// segment starts at an even address, so the little-endian half-word sum needs no rotation.
//
// Work decomposition: thread t of block b owns segments tile_b + t + 256*(u + U*j), u < U, j < J
// (or grid-stride steps when a grid is forced): a wave's loads for one u cover 64 consecutive
// segments (coalesced), each lane has U segments' loads in flight per iteration, and the block's
// tile is contiguous in memory. No pseudo-header (headers only), no cross-lane reduction.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "netcsum_device.h"
#include "netcsum_kernels.h"

namespace netcsum {

namespace {

typedef const __attribute__((address_space(1))) uint32_t gu32;
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef const __attribute__((address_space(1))) u32x2 gu32x2;

template <int ND>
struct Dw {
    uint32_t d[ND];
};

// ND dwords at a 4-B-aligned address: dwordx4 pieces, then x2, then x1.
template <int ND>
__device__ __forceinline__ Dw<ND> load_dw(uintptr_t a) {
    Dw<ND> r;
#pragma unroll
    for (int i = 0; i + 4 <= ND; i += 4) {
        const u32x4 v = *reinterpret_cast<gu32x4*>(a + 4u * (uintptr_t)i);
        r.d[i] = v.x;
        r.d[i + 1] = v.y;
        r.d[i + 2] = v.z;
        r.d[i + 3] = v.w;
    }
    constexpr int b = ND & ~3;
    if constexpr ((ND & 3) >= 2) {
        const u32x2 v = *reinterpret_cast<gu32x2*>(a + 4u * (uintptr_t)b);
        r.d[b] = v.x;
        r.d[b + 1] = v.y;
    }
    if constexpr ((ND & 1) != 0) {
        r.d[ND - 1] = *reinterpret_cast<gu32*>(a + 4u * (uintptr_t)(ND - 1));
    }
    return r;
}

template <int ND, int U>
__global__ void __launch_bounds__(256) seg_small_kernel(SegBatchArgs P) {
    // tile mode (P.tile = J > 0): block b owns segments [b*256*U*J, (b+1)*256*U*J);
    // grid-stride mode (P.tile = 0): block b starts at b*256*U and strides by the grid.
    constexpr uint64_t chunk = 256ull * U;
    const bool tiled = P.tile != 0u;
    const uint64_t first = (tiled ? (uint64_t)blockIdx.x * chunk * P.tile : (uint64_t)blockIdx.x * chunk) + threadIdx.x;
    const uint64_t step = tiled ? chunk : (uint64_t)gridDim.x * chunk;
    const uint64_t lim = tiled ? min((uint64_t)P.n_seg, ((uint64_t)blockIdx.x + 1u) * chunk * P.tile)
                               : (uint64_t)P.n_seg;
    const uintptr_t base = (uintptr_t)P.base;
    const uintptr_t z = zero_addr();
    const uint32_t rem = P.seg_len & 3u;                         // bytes used in the last dword
    const uint32_t last_mask = rem ? ((1u << (8u * rem)) - 1u) : 0xFFFFFFFFu;
    for (uint64_t i0 = first; i0 < lim; i0 += step) {
        Dw<ND> w[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = i0 + 256ull * u;
            w[u] = load_dw<ND>(i < lim ? base + i * P.seg_stride : z);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = i0 + 256ull * u;
            uint32_t acc = 0u;
#pragma unroll
            for (int d = 0; d < ND - 1; ++d) {
                acc = __builtin_amdgcn_sad_u16(w[u].d[d], 0u, acc);
            }
            acc = __builtin_amdgcn_sad_u16(w[u].d[ND - 1] & last_mask, 0u, acc);
            const uint32_t s = fold16(acc);
            if (i < lim) {
                if (P.verify) {
                    static_cast<uint8_t*>(P.out)[i] = (s == 0xFFFFu) ? 1u : 0u;
                } else {
                    static_cast<uint16_t*>(P.out)[i] = (uint16_t)(~s);
                }
            }
        }
    }
}

template <int ND>
hipError_t launch_small_nd(const SegBatchArgs& a, int grid, hipStream_t s) {
    constexpr int U = ND <= 8 ? 4 : 2;
    if (a.tile > 0u || grid <= 0) {                    // tile mode: the grid follows the tiles
        const uint64_t per = 256ull * U * (a.tile ? a.tile : 1u);
        grid = (int)(((uint64_t)a.n_seg + per - 1u) / per);
    }
    hipLaunchKernelGGL((seg_small_kernel<ND, U>), dim3(grid), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace

bool small_supported(const SegBatchArgs& a) {
    return a.seg_off == nullptr && a.pseudo == nullptr && a.seg_len >= 1u && a.seg_len <= 64u &&
           (((uintptr_t)a.base | (uintptr_t)a.seg_stride) & 3u) == 0u;
}

// a.tile > 0 (or grid <= 0): one block per contiguous tile of 256 x U x tile segments;
// a.tile == 0 with grid > 0: grid-stride over that grid.
hipError_t launch_small_batch(const SegBatchArgs& a, int grid, hipStream_t s) {
    switch ((a.seg_len + 3u) >> 2) {
    case 1: return launch_small_nd<1>(a, grid, s);
    case 2: return launch_small_nd<2>(a, grid, s);
    case 3: return launch_small_nd<3>(a, grid, s);
    case 4: return launch_small_nd<4>(a, grid, s);
    case 5: return launch_small_nd<5>(a, grid, s);
    case 6: return launch_small_nd<6>(a, grid, s);
    case 7: return launch_small_nd<7>(a, grid, s);
    case 8: return launch_small_nd<8>(a, grid, s);
    case 9: return launch_small_nd<9>(a, grid, s);
    case 10: return launch_small_nd<10>(a, grid, s);
    case 11: return launch_small_nd<11>(a, grid, s);
    case 12: return launch_small_nd<12>(a, grid, s);
    case 13: return launch_small_nd<13>(a, grid, s);
    case 14: return launch_small_nd<14>(a, grid, s);
    case 15: return launch_small_nd<15>(a, grid, s);
    case 16: return launch_small_nd<16>(a, grid, s);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace netcsum
