// netcsum_chains.hip — batched NET_BUF chain checksums on gfx950.
//
// Chain i = pseudo-header ‖ piece_0 ‖ piece_1 ‖ … (pieces = the per-buffer (DataPtr + ix, len) spans
// NetUtil_16BitOnesCplSumDataCalc resolves, net_util.c:1611-1640; the host helper
// NetUtil_MI355X_ChainToSpans produces them). This is the reference's multi-buffer case: IP
// fragment reassembly chains (net_ipv4.c:6523) and jumbo datagrams, where an odd-length buffer
// carries its dangling octet into the next one (net_util.c:1385-1393, 1463-1471).
//
// Exactness: chains are unbounded in total length, and the reference accumulates per-buffer sums
// into a u32 that wraps (net_util.c:1554, :1685) — mod-65535 arithmetic is NOT exact past 2^32.
// So this kernel computes the EXACT big-endian word sum as 256*E + O, where E / O are the exact sums
// of the bytes at even / odd positions of the chain's stream: per dword, v_sad_u16 of
// (x & 0x00FF00FF) and ((x >> 8) & 0x00FF00FF) gives the even- and odd-ADDRESS byte sums; a piece
// whose stream position parity differs from its address parity swaps the two. The result is
// wrapped to u32 exactly like the reference, then folded.
//
// One G-lane group per chain, pieces in order (their stream offsets are a running sum), chunks of a
// piece spread over the group's lanes. Piece count 0 means pdata_buf == NULL: an odd-length
// pseudo-header then loses its last octet (net_util.c:1601-1611); pass one zero-length piece for a
// chain of empty buffers.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "netcsum_device.h"
#include "netcsum_kernels.h"

namespace netcsum {

namespace {

struct EO {
    uint32_t e;   // bytes at even ADDRESSES (lane partial, exact)
    uint32_t o;   // bytes at odd addresses
};

__device__ __forceinline__ void eo_add(u32x4 v, EO& s) {
    s.e = __builtin_amdgcn_sad_u16(v.x & 0x00FF00FFu, 0u, s.e);
    s.o = __builtin_amdgcn_sad_u16((v.x >> 8) & 0x00FF00FFu, 0u, s.o);
    s.e = __builtin_amdgcn_sad_u16(v.y & 0x00FF00FFu, 0u, s.e);
    s.o = __builtin_amdgcn_sad_u16((v.y >> 8) & 0x00FF00FFu, 0u, s.o);
    s.e = __builtin_amdgcn_sad_u16(v.z & 0x00FF00FFu, 0u, s.e);
    s.o = __builtin_amdgcn_sad_u16((v.z >> 8) & 0x00FF00FFu, 0u, s.o);
    s.e = __builtin_amdgcn_sad_u16(v.w & 0x00FF00FFu, 0u, s.e);
    s.o = __builtin_amdgcn_sad_u16((v.w >> 8) & 0x00FF00FFu, 0u, s.o);
}

// Exact even/odd-address byte sums of [a, a + len) over the group's lanes (this lane's share).
template <int G>
__device__ __forceinline__ EO span_eo(uintptr_t a, uint32_t len, int lane) {
    EO s{0u, 0u};
    const uintptr_t q0 = a & ~(uintptr_t)15;
    const uint32_t lead = (uint32_t)(a & 15u);
    const uint32_t rend = lead + len;
    const uint32_t nch = len ? (rend + 15u) >> 4 : 0u;
    for (uint32_t c = (uint32_t)lane; c < nch; c += (uint32_t)G) {
        u32x4 v = load16<false>(reinterpret_cast<gu32x4*>(q0 + 16u * (uintptr_t)c));
        eo_add(edge_mask_rel(v, c, lead, rend), s);
    }
    return s;
}

template <int G>
__device__ __forceinline__ uint64_t group_sum64(uint64_t v) {
#pragma unroll
    for (int m = G / 2; m >= 1; m >>= 1) {
        v += __shfl_xor(v, m, 64);
    }
    return v;
}

template <int G>
__global__ void __launch_bounds__(256) chain_batch_kernel(ChainBatchArgs A) {
    const int lane = (int)(threadIdx.x & (G - 1));
    const uint32_t gpb = blockDim.x / G;
    for (uint32_t ch = blockIdx.x * gpb + threadIdx.x / G; ch < A.n; ch += gridDim.x * gpb) {
        const uint32_t p0 = A.first[ch], p1 = A.first[ch + 1];
        uint64_t E = 0u, O = 0u;                                  // stream-parity sums (this lane)
        uint32_t spos = 0u;                                       // stream offset parity tracker
        if (A.pseudo && A.pseudo_len) {
            uint32_t plen = A.pseudo_len;
            if (p0 == p1 && (plen & 1u)) {
                plen -= 1u;                                       // NULL chain quirk
            }
            const uintptr_t pa = (uintptr_t)A.pseudo + (uint64_t)ch * A.pseudo_stride;
            const EO s = span_eo<G>(pa, plen, lane);
            if (pa & 1u) { E += s.o; O += s.e; } else { E += s.e; O += s.o; }
            spos = A.pseudo_len & 1u;                             // later pieces follow ALL pseudo bytes
        }
        for (uint32_t j = p0; j < p1; ++j) {
            const uintptr_t a = (uintptr_t)A.base + A.off[j];
            const uint32_t len = A.len[j];
            const EO s = span_eo<G>(a, len, lane);
            if (((uint32_t)(a & 1u)) != spos) { E += s.o; O += s.e; } else { E += s.e; O += s.o; }
            spos ^= (len & 1u);
        }
        E = group_sum64<G>(E);
        O = group_sum64<G>(O);
        if (lane == 0) {
            uint32_t sum = (uint32_t)((E << 8) + O);              // the reference's u32 accumulator
            while (sum >> 16) {
                sum = (sum & 0xFFFFu) + (sum >> 16);
            }
            const uint32_t host = ((sum & 0xFFu) << 8) | (sum >> 8);   // NET_UTIL_NET_TO_HOST_16
            if (A.verify) {
                static_cast<uint8_t*>(A.out)[ch] = (host == 0xFFFFu) ? 1u : 0u;
            } else {
                static_cast<uint16_t*>(A.out)[ch] = (uint16_t)(~host);
            }
        }
    }
}

}  // namespace

hipError_t launch_chain_batch(const ChainBatchArgs& a, int group, int grid, hipStream_t s) {
    switch (group) {
    case 16:
        hipLaunchKernelGGL(chain_batch_kernel<16>, dim3(grid), dim3(256), 0, s, a);
        break;
    case 32:
        hipLaunchKernelGGL(chain_batch_kernel<32>, dim3(grid), dim3(256), 0, s, a);
        break;
    default:
        hipLaunchKernelGGL(chain_batch_kernel<64>, dim3(grid), dim3(256), 0, s, a);
        break;
    }
    return hipGetLastError();
}

}  // namespace netcsum
