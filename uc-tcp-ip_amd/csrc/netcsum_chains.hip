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
// Two forms. chain_wave_kernel (default): one WAVE per chain, 16 lanes per piece, four pieces of the
// chain per step, six 16-B chunks per lane per pass (one pass covers a 1480-B fragment at any
// alignment), two steps in flight — step t+1's loads are issued before step t is reduced. The four
// piece descriptors of a step are wave-uniform, so they are scalar loads issued a step ahead, and a
// piece's stream parity (pseudo-header length plus the lengths before it, mod 2) is SALU arithmetic
// on them. chain_batch_kernel<G> (tuning option): a G-lane group per chain, pieces in order, one load
// per lane in flight. Piece count 0 means pdata_buf == NULL: an odd-length pseudo-header then loses
// its last octet (net_util.c:1601-1611); pass one zero-length piece for a chain of empty buffers.
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

__device__ __forceinline__ void chain_out(const ChainBatchArgs& A, uint32_t ch, uint64_t E, uint64_t O) {
    uint32_t sum = (uint32_t)((E << 8) + O);                      // the reference's u32 accumulator
    while (sum >> 16) {
        sum = (sum & 0xFFFFu) + (sum >> 16);
    }
    const uint32_t host = ((sum & 0xFFu) << 8) | (sum >> 8);       // NET_UTIL_NET_TO_HOST_16
    if (A.verify) {
        static_cast<uint8_t*>(A.out)[ch] = (host == 0xFFFFu) ? 1u : 0u;
    } else {
        static_cast<uint16_t*>(A.out)[ch] = (uint16_t)(~host);
    }
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
            chain_out(A, ch, E, O);
        }
    }
}

// ---- chain_wave_kernel ------------------------------------------------------------------------
constexpr int kWQ = 16;    // lanes per piece (quarter of the wave)
constexpr int kWK = 6;     // 16-B chunks per lane per pass

typedef const __attribute__((address_space(4))) uint64_t c_u64;    // constant address space:
typedef const __attribute__((address_space(4))) uint32_t c_u32;    // scalar loads when uniform

struct StepDesc {           // the four pieces of one step (len 0 past the chain's end)
    uint64_t off[4];
    uint32_t len[4];
};

__device__ __forceinline__ StepDesc step_desc(const ChainBatchArgs& A, uint32_t j0, uint32_t p1) {
    StepDesc d;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t j = j0 + (uint32_t)q;
        d.off[q] = 0u;
        d.len[q] = 0u;
        if (j < p1) {
            d.off[q] = *reinterpret_cast<c_u64*>(reinterpret_cast<uintptr_t>(A.off + j));
            const uintptr_t la = reinterpret_cast<uintptr_t>(A.len + j);
            const uint32_t w = *reinterpret_cast<c_u32*>(la & ~(uintptr_t)3);
            d.len[q] = (w >> (8u * (uint32_t)(la & 2u))) & 0xFFFFu;
        }
    }
    return d;
}

__device__ __forceinline__ uint32_t step_odd(const StepDesc& d) {
    return (d.len[0] ^ d.len[1] ^ d.len[2] ^ d.len[3]) & 1u;
}

struct WStage {
    u32x4     v[kWK];
    uintptr_t a;           // piece start
    uint32_t  len;
    uint32_t  swap;        // 1: the piece's stream parity differs from its address parity
};

// Issue quarter qi's piece of the step described by d; par = stream parity at the step's first piece.
__device__ __forceinline__ void wave_issue(WStage& st, const StepDesc& d, uint32_t par, uintptr_t base, int qi,
                                           int ql) {
    const uint32_t o0 = d.len[0] & 1u, o1 = d.len[1] & 1u, o2 = d.len[2] & 1u;
    uint64_t off = d.off[0];
    uint32_t len = d.len[0], pre = 0u;
    if (qi == 1) { off = d.off[1]; len = d.len[1]; pre = o0; }
    if (qi == 2) { off = d.off[2]; len = d.len[2]; pre = o0 ^ o1; }
    if (qi == 3) { off = d.off[3]; len = d.len[3]; pre = o0 ^ o1 ^ o2; }
    const uintptr_t a = base + off;
    st.a = a;
    st.len = len;
    st.swap = ((uint32_t)(a & 1u)) ^ par ^ pre;
    const uintptr_t q0 = a & ~(uintptr_t)15;
    const uint32_t nch = len ? (uint32_t)(((a & 15u) + len + 15u) >> 4) : 0u;
    const uintptr_t z = zero_addr();
#pragma unroll
    for (int k = 0; k < kWK; ++k) {
        const uint32_t c = (uint32_t)(k * kWQ + ql);
        st.v[k] = load16<true>(reinterpret_cast<gu32x4*>((c < nch) ? (q0 + 16u * (uintptr_t)c) : z));
    }
}

__device__ __forceinline__ void wave_consume(const WStage& st, int ql, uint64_t& E, uint64_t& O) {
    const uint32_t lead = (uint32_t)(st.a & 15u);
    const uint32_t rend = lead + st.len;
    const uint32_t nch = st.len ? (rend + 15u) >> 4 : 0u;
    EO s{0u, 0u};
#pragma unroll
    for (int k = 0; k < kWK; ++k) {
        // every loaded register consumed on every path (netcsum_device.h, opaque)
        const uint32_t c = (uint32_t)(k * kWQ + ql);
        const uint32_t keep = (c < nch) ? 0xFFFFFFFFu : 0u;
        u32x4 v = opaque(st.v[k]);
        v.x &= keep; v.y &= keep; v.z &= keep; v.w &= keep;
        if (c < nch) {
            v = edge_mask_rel(v, c, lead, rend);
        }
        eo_add(v, s);
    }
    if (nch > (uint32_t)(kWQ * kWK)) {                            // pieces longer than one pass
        const uintptr_t q0 = st.a & ~(uintptr_t)15;
        for (uint32_t c0 = (uint32_t)(kWQ * kWK); c0 < nch; c0 += (uint32_t)(kWQ * kWK)) {
            u32x4 w[kWK];
#pragma unroll
            for (int k = 0; k < kWK; ++k) {
                const uint32_t c = c0 + (uint32_t)(k * kWQ + ql);
                w[k] = load16<true>(reinterpret_cast<gu32x4*>((c < nch) ? (q0 + 16u * (uintptr_t)c) : zero_addr()));
            }
#pragma unroll
            for (int k = 0; k < kWK; ++k) {
                const uint32_t c = c0 + (uint32_t)(k * kWQ + ql);
                u32x4 v = w[k];
                if (c < nch) {
                    v = edge_mask_rel(v, c, lead, rend);
                }
                eo_add(v, s);
            }
        }
    }
    if (st.swap) { E += s.o; O += s.e; } else { E += s.e; O += s.o; }
}

__global__ void __launch_bounds__(256) chain_wave_kernel(ChainBatchArgs A) {
    const int lane = (int)(threadIdx.x & 63u);
    const int ql = lane & (kWQ - 1);
    const int qi = lane >> 4;
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t nw = gridDim.x * 4u;
    const uintptr_t base = (uintptr_t)A.base;
    for (uint32_t ch = blockIdx.x * 4u + w; ch < A.n; ch += nw) {      // wave-uniform
        const uint32_t p0 = *reinterpret_cast<c_u32*>(reinterpret_cast<uintptr_t>(A.first + ch));
        const uint32_t p1 = *reinterpret_cast<c_u32*>(reinterpret_cast<uintptr_t>(A.first + ch + 1u));
        uint64_t E = 0u, O = 0u;
        uint32_t par = 0u;                                        // stream parity at the next piece
        if (A.pseudo && A.pseudo_len) {
            uint32_t plen = A.pseudo_len;
            if (p0 == p1 && (plen & 1u)) {
                plen -= 1u;                                       // NULL chain quirk
            }
            const uintptr_t pa = (uintptr_t)A.pseudo + (uint64_t)ch * A.pseudo_stride;
            const EO s = span_eo<64>(pa, plen, lane);
            if (pa & 1u) { E += s.o; O += s.e; } else { E += s.e; O += s.o; }
            par = A.pseudo_len & 1u;                              // pieces follow ALL pseudo bytes
        }
        const uint32_t steps = (p1 - p0 + 3u) >> 2;
        if (steps != 0u) {
            WStage S0, S1;
            StepDesc d = step_desc(A, p0, p1);
            wave_issue(S0, d, par, base, qi, ql);
            par ^= step_odd(d);
            d = step_desc(A, p0 + 4u, p1);
            for (uint32_t t = 0; t < steps; t += 2u) {
                wave_issue(S1, d, par, base, qi, ql);             // step t + 1 (empty past the end)
                par ^= step_odd(d);
                d = step_desc(A, p0 + 4u * (t + 2u), p1);
                wave_consume(S0, ql, E, O);                       // step t
                wave_issue(S0, d, par, base, qi, ql);             // step t + 2
                par ^= step_odd(d);
                d = step_desc(A, p0 + 4u * (t + 3u), p1);
                wave_consume(S1, ql, E, O);                       // step t + 1
            }
        }
        E = group_sum64<64>(E);
        O = group_sum64<64>(O);
        if (lane == 0) {
            chain_out(A, ch, E, O);
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
    case 64:
        hipLaunchKernelGGL(chain_batch_kernel<64>, dim3(grid), dim3(256), 0, s, a);
        break;
    default:
        hipLaunchKernelGGL(chain_wave_kernel, dim3(grid), dim3(256), 0, s, a);
        break;
    }
    return hipGetLastError();
}

}  // namespace netcsum
