// netcsum_kernels.hip — gfx950 (MI355X / CDNA4) kernels of the Internet-checksum path.
//
// Replaces the inner loops of µC/TCP-IP V3.06.01 Source/net_util.c:
//   NetUtil_16BitSumDataCalc   :1321-1475  (32-bit word loop :1423-1435, odd-octet carry :1385-1393,
//                                           :1463-1471)
//   NetUtil_16BitSumHdrCalc    :1160-1208
//   the end-around-carry folds :184-186, :271-273, :1690-1692
// and the optional native-loop seam NetUtil_16BitSumDataCalcAlign_32 (net_util.h:486-490,
// Ports/ARM/GNU/net_util_a.s:108-182), whose ROR#8 trick is the same byte-order independence
// these kernels use (RFC 1071 §2(B)).
//
// Arithmetic (all integer, bit-exact; no MFMA — this is an HBM-bound byte sum):
//   * Bytes are read as little-endian dwords in an ABSOLUTE 16-byte-aligned frame (dwordx4
//     loads, 1 KiB per wave-instruction). v_sad_u16(x, 0, acc) adds both 16-bit halves of a
//     dword into a 32-bit lane accumulator in ONE VALU op. In that frame a byte at an even
//     address carries weight 1 and a byte at an odd address weight 256 (mod 65535).
//   * A span whose first byte sits at an odd position of the checksummed stream (odd address, or
//     after an odd-length pseudo-header) is corrected by rotating its folded 16-bit partial by
//     8 bits (x*256 mod 65535) — the reference's prepend/carry of the odd octet.
//   * Little-endian word sums fold to bswap16 of the reference's big-endian fold, so the
//     reference's host-order return value NET_TO_HOST_16(~fold_be) is simply ~fold_le.
//   * End-around-carry adds keep "zero iff every byte is zero" (the 0x0000 vs 0xFFFF distinction
//     of the reference's fold) for any reduction tree.
//   * Per-segment totals (pseudo <= 65535 B + segment <= 65535 B, CPU_INT16U lengths as in the
//     reference) never exceed 2^32 as exact big-endian sums, so mod-65535 arithmetic equals the
//     reference's u32 accumulate-then-fold exactly.
//
// Work decomposition: a GROUP of G lanes (G = 1…64, a divisor of the 64-lane wave) owns one
// segment at a time; each lane streams K 16-byte chunks of the segment per pass (all K loads in
// flight before the first add), masks the partial chunks at the segment edges, and the group
// folds its lane partials with cross-lane shuffles. Groups grid-stride over segments.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "netcsum_kernels.h"

namespace netcsum {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
// Global-address-space view: addresses are computed as integers (absolute 16-B frame), and an
// explicit addrspace(1) pointer keeps the loads on global_load_* (not flat_load_*, which would
// also count on lgkmcnt and add a flat-aperture check).
typedef const __attribute__((address_space(1))) u32x4 gu32x4;

__device__ __forceinline__ uint32_t fold16(uint32_t s) {
    s = (s & 0xFFFFu) + (s >> 16);
    s = (s & 0xFFFFu) + (s >> 16);
    return s;                                   // in [0, 0xFFFF]; 0 iff the input was 0
}

__device__ __forceinline__ uint32_t rot8(uint32_t s16) {   // x * 256 mod 65535 on a 16-bit value
    return ((s16 << 8) | (s16 >> 8)) & 0xFFFFu;
}

template <bool NT>
__device__ __forceinline__ u32x4 load16(gu32x4* p) {
    if constexpr (NT) {
        return __builtin_nontemporal_load(p);
    } else {
        return *p;
    }
}

__device__ __forceinline__ uint32_t sum4(u32x4 v, uint32_t acc) {
    acc = __builtin_amdgcn_sad_u16(v.x, 0u, acc);
    acc = __builtin_amdgcn_sad_u16(v.y, 0u, acc);
    acc = __builtin_amdgcn_sad_u16(v.z, 0u, acc);
    acc = __builtin_amdgcn_sad_u16(v.w, 0u, acc);
    return acc;
}

// Keep bytes [lo, hi) of a dword whose first byte is byte `base` of its chunk.
__device__ __forceinline__ uint32_t dword_mask(int lo, int hi, int base) {
    int l = min(max(lo - base, 0), 4);
    int h = min(max(hi - base, 0), 4);
    uint32_t mh = (h >= 4) ? 0xFFFFFFFFu : ((1u << (8 * h)) - 1u);
    uint32_t ml = (l >= 4) ? 0u : (0xFFFFFFFFu << (8 * l));
    return mh & ml;
}

__device__ __forceinline__ u32x4 mask_chunk(u32x4 v, int lo, int hi) {
    v.x &= dword_mask(lo, hi, 0);
    v.y &= dword_mask(lo, hi, 4);
    v.z &= dword_mask(lo, hi, 8);
    v.w &= dword_mask(lo, hi, 12);
    return v;
}

// Sum (in the absolute LE frame) of the byte span [a, a+len) by the G lanes of a group; K chunks
// per lane per pass. Returns the lane's 32-bit partial.
template <int G, int K, bool NT>
__device__ __forceinline__ uint32_t span_partial(uintptr_t a, uint32_t len, int lane) {
    const uintptr_t q0  = a & ~(uintptr_t)15;
    const uintptr_t end = a + len;
    const uint32_t  nch = len ? (uint32_t)((end - q0 + 15) >> 4) : 0u;
    const int       lead = (int)(a - q0);
    uint32_t acc = 0u;
    for (uint32_t c0 = 0; c0 < nch; c0 += (uint32_t)(G * K)) {
        u32x4 v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t c = c0 + (uint32_t)(k * G + lane);
            v[k] = (c < nch) ? load16<NT>(reinterpret_cast<gu32x4*>(q0 + 16u * (uintptr_t)c))
                             : u32x4{0u, 0u, 0u, 0u};
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t c = c0 + (uint32_t)(k * G + lane);
            const uintptr_t q = q0 + 16u * (uintptr_t)c;
            const int lo = (c == 0u) ? lead : 0;
            const int hi = (c < nch && q + 16u > end) ? (int)(end - q) : 16;
            if (lo != 0 || hi != 16) {
                v[k] = mask_chunk(v[k], lo, hi);
            }
            acc = sum4(v[k], acc);
        }
    }
    return acc;
}

template <int G>
__device__ __forceinline__ uint32_t group_sum(uint32_t s) {
#pragma unroll
    for (int m = G / 2; m >= 1; m >>= 1) {
        s += __shfl_xor(s, m, 64);
    }
    return s;
}

// ---------------------------------------------------------------------------------------------
// Segment batch kernel. out[i] per NETCSUM_OP (include/netcsum_mi355x.h (2)).
// ---------------------------------------------------------------------------------------------
template <int G, int K, bool VARLEN, bool NT>
__global__ void __launch_bounds__(256) seg_batch_kernel(SegBatchArgs P) {
    const int      lane   = (int)(threadIdx.x & (G - 1));
    const uint32_t gpb    = blockDim.x / G;
    const uint32_t step   = gridDim.x * gpb;
    const bool     has_ph = (P.pseudo != nullptr) && (P.pseudo_len != 0u);
    const bool     ph_odd = (P.pseudo_len & 1u) != 0u;

    for (uint32_t seg = blockIdx.x * gpb + threadIdx.x / G; seg < P.n_seg; seg += step) {
        uint64_t off;
        uint32_t len;
        if constexpr (VARLEN) {
            off = P.seg_off[seg];
            len = P.seg_len_v[seg];
        } else {
            off = (uint64_t)seg * P.seg_stride;
            len = P.seg_len;
        }
        const uintptr_t a = (uintptr_t)P.base + off;

        uint32_t s = fold16(span_partial<G, K, NT>(a, len, lane));
        if (((a & 1u) != 0u) != ph_odd) {       // segment starts at an odd stream position
            s = rot8(s);
        }
        if (has_ph) {                            // pseudo-header at stream position 0
            const uintptr_t pa = (uintptr_t)P.pseudo + (uint64_t)seg * P.pseudo_stride;
            uint32_t ps = fold16(span_partial<G, 1, false>(pa, P.pseudo_len, lane));
            if (pa & 1u) {
                ps = rot8(ps);
            }
            s += ps;
        }
        s = fold16(group_sum<G>(s));
        if (lane == 0) {
            if (P.verify) {
                static_cast<uint8_t*>(P.out)[seg] = (s == 0xFFFFu) ? 1u : 0u;
            } else {
                static_cast<uint16_t*>(P.out)[seg] = (uint16_t)(~s);
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Exact big-endian stream sum (host per-packet path): *sum += Σ BE 16-bit words of
// [p, p + n16*16). The stream is staged 16-byte aligned and zero padded by the host, so stream
// position == address and the pad adds nothing. v_perm_b32 swaps the bytes of both halves, then
// v_sad_u16 adds the two big-endian words: exact, no modular folding (the u32 wrap of the
// reference's cross-buffer `sum` is applied by the caller).
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) stream_exact_kernel(gu32x4* __restrict__ p, uint32_t n16,
                                                           unsigned long long* __restrict__ sum) {
    __shared__ unsigned long long wsum[4];
    uint32_t acc = 0u;
    for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < n16; c += gridDim.x * blockDim.x) {
        const u32x4 v = p[c];
        acc = __builtin_amdgcn_sad_u16(__builtin_amdgcn_perm(v.x, v.x, 0x02030001u), 0u, acc);
        acc = __builtin_amdgcn_sad_u16(__builtin_amdgcn_perm(v.y, v.y, 0x02030001u), 0u, acc);
        acc = __builtin_amdgcn_sad_u16(__builtin_amdgcn_perm(v.z, v.z, 0x02030001u), 0u, acc);
        acc = __builtin_amdgcn_sad_u16(__builtin_amdgcn_perm(v.w, v.w, 0x02030001u), 0u, acc);
    }
    unsigned long long w = acc;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        w += __shfl_xor(w, m, 64);
    }
    if ((threadIdx.x & 63u) == 0u) {
        wsum[threadIdx.x >> 6] = w;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0ull;
        for (uint32_t i = 0; i < (blockDim.x >> 6); ++i) {
            t += wsum[i];
        }
        atomicAdd(sum, t);
    }
}

// ---------------------------------------------------------------------------------------------
// Synthetic input (== Oracle_Fill): 8 bytes per splitmix64 call, byte k from word k >> 3.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ uint64_t fill_word(uint64_t w, uint64_t seed, int pattern) {
    switch (pattern) {
    case 1:  return 0ull;
    case 2:  return ~0ull;
    case 3:  return 0x0100FFFF0100FFFFull;      // bytes FF FF 00 01 FF FF 00 01 (period 4 | 8)
    default: return splitmix64(seed + w);
    }
}

// The 8 stream bytes starting at global byte g (any alignment), little-endian packed.
__device__ __forceinline__ uint64_t fill_bytes8(uint64_t g, uint64_t seed, int pattern) {
    const uint32_t r = (uint32_t)(g & 7u);
    const uint64_t lo = fill_word(g >> 3, seed, pattern);
    if (r == 0u) return lo;
    const uint64_t hi = fill_word((g >> 3) + 1u, seed, pattern);
    return (lo >> (8u * r)) | (hi << (64u - 8u * r));
}

// buf must be 8-byte aligned; full 8-byte words are stored as u64, the tail byte-wise.
__global__ void __launch_bounds__(256) fill_kernel(uint8_t* __restrict__ buf, uint64_t n_bytes,
                                                   uint64_t first_byte, uint64_t seed, int pattern) {
    const uint64_t nw = n_bytes >> 3;
    uint64_t* bw = reinterpret_cast<uint64_t*>(buf);
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nw;
         w += (uint64_t)gridDim.x * blockDim.x) {
        bw[w] = fill_bytes8(first_byte + 8u * w, seed, pattern);
    }
    if (blockIdx.x == 0 && threadIdx.x < (n_bytes & 7u)) {
        const uint64_t k = (nw << 3) + threadIdx.x;
        buf[k] = (uint8_t)fill_bytes8(first_byte + k, seed, pattern);
    }
}

// ---------------------------------------------------------------------------------------------
// Roofline probe: pure 16-B/lane HBM read stream (same loads as the checksum kernels, no masks).
// ---------------------------------------------------------------------------------------------
template <bool NT>
__global__ void __launch_bounds__(256) read_stream_kernel(gu32x4* __restrict__ p, uint64_t n16,
                                                          unsigned long long* __restrict__ sink) {
    uint32_t acc = 0u;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; c + 3 * stride < n16; c += 4 * stride) {
        const u32x4 v0 = load16<NT>(p + c);
        const u32x4 v1 = load16<NT>(p + c + stride);
        const u32x4 v2 = load16<NT>(p + c + 2 * stride);
        const u32x4 v3 = load16<NT>(p + c + 3 * stride);
        acc = sum4(v0, acc);
        acc = sum4(v1, acc);
        acc = sum4(v2, acc);
        acc = sum4(v3, acc);
    }
    for (; c < n16; c += stride) {
        acc = sum4(load16<NT>(p + c), acc);
    }
    if (acc == 0x5EEDF00Du) {                  // practically never: keeps the loads alive
        atomicAdd(sink, 1ull);
    }
}

}  // namespace netcsum

// ================================== host-side launchers ===================================

namespace netcsum {

template <int G, int K, bool VARLEN, bool NT>
static hipError_t launch_seg(const SegBatchArgs& a, int grid, int block, hipStream_t s) {
    hipLaunchKernelGGL((seg_batch_kernel<G, K, VARLEN, NT>), dim3(grid), dim3(block), 0, s, a);
    return hipGetLastError();
}

template <int G, int K, bool VARLEN>
static hipError_t launch_seg_nt(const SegBatchArgs& a, int grid, int block, bool nt, hipStream_t s) {
    return nt ? launch_seg<G, K, VARLEN, true>(a, grid, block, s)
              : launch_seg<G, K, VARLEN, false>(a, grid, block, s);
}

template <int G, bool VARLEN>
static hipError_t launch_seg_k(const SegBatchArgs& a, int k, int grid, int block, bool nt, hipStream_t s) {
    switch (k) {
    case 1:  return launch_seg_nt<G, 1, VARLEN>(a, grid, block, nt, s);
    case 2:  return launch_seg_nt<G, 2, VARLEN>(a, grid, block, nt, s);
    case 3:  return launch_seg_nt<G, 3, VARLEN>(a, grid, block, nt, s);
    default: return launch_seg_nt<G, 4, VARLEN>(a, grid, block, nt, s);
    }
}

template <bool VARLEN>
static hipError_t launch_seg_g(const SegBatchArgs& a, int g, int k, int grid, int block, bool nt,
                               hipStream_t s) {
    switch (g) {
    case 1:  return launch_seg_k<1, VARLEN>(a, k, grid, block, nt, s);
    case 4:  return launch_seg_k<4, VARLEN>(a, k, grid, block, nt, s);
    case 8:  return launch_seg_k<8, VARLEN>(a, k, grid, block, nt, s);
    case 16: return launch_seg_k<16, VARLEN>(a, k, grid, block, nt, s);
    case 32: return launch_seg_k<32, VARLEN>(a, k, grid, block, nt, s);
    default: return launch_seg_k<64, VARLEN>(a, k, grid, block, nt, s);
    }
}

hipError_t launch_seg_batch(const SegBatchArgs& a, const LaunchCfg& c, hipStream_t s) {
    return a.seg_off ? launch_seg_g<true>(a, c.group_lanes, c.chunks_per_pass, c.grid, c.block, c.nt, s)
                     : launch_seg_g<false>(a, c.group_lanes, c.chunks_per_pass, c.grid, c.block, c.nt, s);
}

hipError_t launch_stream_exact(const void* d_p, uint32_t n16, unsigned long long* d_sum, int grid,
                               hipStream_t s) {
    hipLaunchKernelGGL(stream_exact_kernel, dim3(grid), dim3(256), 0, s,
                       reinterpret_cast<gu32x4*>(reinterpret_cast<uintptr_t>(d_p)), n16, d_sum);
    return hipGetLastError();
}

hipError_t launch_fill(void* d_buf, uint64_t n_bytes, uint64_t first_byte, uint64_t seed, int pattern, int grid,
                       hipStream_t s) {
    hipLaunchKernelGGL(fill_kernel, dim3(grid), dim3(256), 0, s, static_cast<uint8_t*>(d_buf), n_bytes,
                       first_byte, seed, pattern);
    return hipGetLastError();
}

hipError_t launch_read_stream(const void* d_p, uint64_t n16, unsigned long long* d_sink, int grid, bool nt,
                              hipStream_t s) {
    if (nt) {
        hipLaunchKernelGGL(read_stream_kernel<true>, dim3(grid), dim3(256), 0, s,
                           reinterpret_cast<gu32x4*>(reinterpret_cast<uintptr_t>(d_p)), n16, d_sink);
    } else {
        hipLaunchKernelGGL(read_stream_kernel<false>, dim3(grid), dim3(256), 0, s,
                           reinterpret_cast<gu32x4*>(reinterpret_cast<uintptr_t>(d_p)), n16, d_sink);
    }
    return hipGetLastError();
}

}  // namespace netcsum
