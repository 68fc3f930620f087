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

#include <algorithm>

#include "netcsum_device.h"
#include "netcsum_kernels.h"
#include "netcsum_stream.h"

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

// Chain `ch` (wave-uniform) by the calling wave.
__device__ __forceinline__ void wave_chain(const ChainBatchArgs& A, uint32_t ch) {
    const int lane = (int)(threadIdx.x & 63u);
    const int ql = lane & (kWQ - 1);
    const int qi = lane >> 4;
    const uintptr_t base = (uintptr_t)A.base;
    {
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

__global__ void __launch_bounds__(256) chain_wave_kernel(ChainBatchArgs A) {
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t nw = gridDim.x * 4u;
    for (uint32_t ch = blockIdx.x * 4u + w; ch < A.n; ch += nw) {      // wave-uniform
        wave_chain(A, ch);
    }
}

// ---- two-pass form (default) --------------------------------------------------------------------
// The wave-per-chain kernel reads a 64-KiB-datagram batch (16 Ki chains x 45 fragments of 1480 B) in
// 0.195 ms; the segment kernel in its lane-group form, 16 lanes x 6 chunks per segment, two segments
// in flight per group, blocks owning tiles of 64 consecutive segments, reads the same fragments as
// a varlen batch in 0.165 ms (profiles/r3s_frag_stream_probe.jsonl; 0.173 without the tiles). So
// chain batches take two passes:
//  1. chain_piece_kernel, that segment form over the batch's pieces in index order: per piece the
//     exact sums of its bytes at even / odd ADDRESSES (taken as a byte sum and a half-word sum, two
//     VALU ops per dword) into an 8-B record;
//  2. chain_combine_kernel, a wave per chain, 64 pieces per step: each piece's stream parity
//     (pseudo-header length + the lengths before it, mod 2) from a ballot of the odd lengths, the
//     record swapped where that differs from the address parity, the pseudo-header added, the
//     exact 64-bit total wrapped to u32 like the reference accumulator and folded (chain_out).
// The piece count lives on the device (chain_first[n]); the records go to a scratch buffer of `cap`
// pieces sized by the host from the chain count, and a batch with more pieces than that is done by
// the combine kernel in the wave-per-chain form (pass 1 then returns at once) — correct, slower.
constexpr int kPG = 16;    // lanes per piece
constexpr int kPK = 6;     // 16-B chunks per lane per pass
constexpr uint32_t kPTile = 4u;   // pieces per group per tile (a block's tile: 64 consecutive pieces)

struct PieceStage {
    u32x4     v[kPK];
    uintptr_t a;
    uint32_t  len;
};

__device__ __forceinline__ void piece_issue(PieceStage& st, uintptr_t a, uint32_t len, int lane) {
    st.a = a;
    st.len = len;
    const uintptr_t q0 = a & ~(uintptr_t)15;
    const uint32_t nch = len ? (uint32_t)(((a & 15u) + len + 15u) >> 4) : 0u;
    const uintptr_t z = zero_addr();
#pragma unroll
    for (int k = 0; k < kPK; ++k) {
        const uint32_t c = (uint32_t)(k * kPG + lane);
        st.v[k] = load16<true>(reinterpret_cast<gu32x4*>((c < nch) ? (q0 + 16u * (uintptr_t)c) : z));
    }
}

// Byte sum b and little-endian half-word sum h (= e + 256 o) of this lane's share of the piece.
__device__ __forceinline__ void piece_consume(const PieceStage& st, int lane, uint32_t& b, uint32_t& h) {
    const uint32_t lead = (uint32_t)(st.a & 15u);
    const uint32_t rend = lead + st.len;
    const uint32_t nch = st.len ? (rend + 15u) >> 4 : 0u;
    b = 0u;
    h = 0u;
    auto add = [&](u32x4 v) {
        b = __builtin_amdgcn_sad_u8(v.x, 0u, b);
        h = __builtin_amdgcn_sad_u16(v.x, 0u, h);
        b = __builtin_amdgcn_sad_u8(v.y, 0u, b);
        h = __builtin_amdgcn_sad_u16(v.y, 0u, h);
        b = __builtin_amdgcn_sad_u8(v.z, 0u, b);
        h = __builtin_amdgcn_sad_u16(v.z, 0u, h);
        b = __builtin_amdgcn_sad_u8(v.w, 0u, b);
        h = __builtin_amdgcn_sad_u16(v.w, 0u, h);
    };
#pragma unroll
    for (int k = 0; k < kPK; ++k) {
        const uint32_t c = (uint32_t)(k * kPG + lane);
        u32x4 v = opaque(st.v[k]);
        if (c < nch) {
            v = edge_mask_rel(v, c, lead, rend);
        }
        add(v);
    }
    if (nch > (uint32_t)(kPG * kPK)) {                            // pieces longer than one pass
        const uintptr_t q0 = st.a & ~(uintptr_t)15;
        for (uint32_t c0 = (uint32_t)(kPG * kPK); c0 < nch; c0 += (uint32_t)(kPG * kPK)) {
            u32x4 w[kPK];
#pragma unroll
            for (int k = 0; k < kPK; ++k) {
                const uint32_t c = c0 + (uint32_t)(k * kPG + lane);
                w[k] = load16<true>(reinterpret_cast<gu32x4*>((c < nch) ? (q0 + 16u * (uintptr_t)c) : zero_addr()));
            }
#pragma unroll
            for (int k = 0; k < kPK; ++k) {
                const uint32_t c = c0 + (uint32_t)(k * kPG + lane);
                u32x4 v = w[k];
                if (c < nch) {
                    v = edge_mask_rel(v, c, lead, rend);
                }
                add(v);
            }
        }
    }
}

// Group-reduce (b, h) and store the piece's record (e | o << 32); h - b = 255 o exactly (a piece
// is < 64 KiB, so o < 2^24), divided by multiplying with 255's inverse mod 2^32.
__device__ __forceinline__ void piece_store(uint64_t* eo, uint32_t j, uint32_t b, uint32_t h, int lane, bool valid) {
#pragma unroll
    for (int m = kPG / 2; m >= 1; m >>= 1) {
        b += (uint32_t)__shfl_xor((int)b, m, 64);
        h += (uint32_t)__shfl_xor((int)h, m, 64);
    }
    if (valid && lane == 0) {
        const uint32_t o = (h - b) * 0xFEFEFEFFu;
        eo[j] = (uint64_t)(b - o) | ((uint64_t)o << 32);
    }
}

// BAL (NETCSUM_TUNE_CHAIN_GRID >= 1, round 6): a grid of whole multiples of the resident blocks, block b
// owning the contiguous pieces [np b / grid, np (b + 1) / grid) — every group the same piece count
// within one, no block starting late, the descriptors prefetched across what were tile boundaries —
// group g taking pieces lo + g + 16 i. Otherwise one tile of 64 consecutive pieces per block.
// TOUCH (NETCSUM_TUNE_STREAM_TOUCH 1): the row touch of the stream kernels (netcsum_stream.h) for a
// group's first 4 pieces — lanes 0..7 load one dword, plain policy, at +0 / +1 KiB of piece l / 2 with
// the first data loads, never used — so the pieces the group streams later have requests under way.
template <bool BAL, bool TOUCH>
__global__ void __launch_bounds__(256) chain_piece_kernel(ChainBatchArgs A, uint64_t* eo, uint32_t cap) {
    const int lane = (int)(threadIdx.x & (kPG - 1));
    constexpr uint32_t gpb = 256u / kPG;                          // groups per block
    constexpr uint32_t tile = gpb * kPTile;                       // pieces per block tile
    const uint32_t g = threadIdx.x / kPG;
    const uint32_t np = *reinterpret_cast<c_u32*>(reinterpret_cast<uintptr_t>(A.first + A.n));
    const uint32_t ntiles = (np + tile - 1u) / tile;
    if (np > cap) {                                               // no room for the records: the
        return;                                                   // combine pass does the batch
    }
    uint32_t bid, iters, lo = 0u, lim = np;
    if constexpr (BAL) {
        bid = A.xcd ? sv::xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
        lo = (uint32_t)(((uint64_t)np * bid) / gridDim.x);
        lim = (uint32_t)(((uint64_t)np * (bid + 1u)) / gridDim.x);
        iters = (lim - lo + gpb - 1u) / gpb;                      // block-uniform
        iters += iters & 1u;                                      // (the loop takes two at a time)
        if (iters == 0u) {
            return;
        }
    } else {
        if (blockIdx.x >= ntiles) {
            return;
        }
        // this block's tiles: bid, + gridDim.x, ...; group g takes pieces tile*64 + g + 16 k. With one
        // tile per block (the default grid), the XCD-aware order: the blocks the dispatcher places on one
        // XCD take one contiguous 1/8 of the tiles (sv::xcd_block over the first ntiles blocks, which
        // are the ones with a tile), as the segment stream kernels' runs do
        bid = (A.xcd && ntiles <= gridDim.x) ? sv::xcd_block(blockIdx.x, ntiles, A.xcd) : blockIdx.x;
        iters = ((ntiles - bid + gridDim.x - 1u) / gridDim.x) * kPTile;   // block-uniform
    }
    auto piece_at = [&](uint32_t i) -> uint32_t {                 // the group's i-th piece
        if constexpr (BAL) {
            return lo + g + gpb * i;
        } else {
            return (bid + (i / kPTile) * gridDim.x) * tile + g + gpb * (i % kPTile);
        }
    };
    const uintptr_t base = (uintptr_t)A.base;
    auto desc = [&](uint32_t j, uint64_t& off, uint32_t& len) {
        const uint32_t jc = j < lim ? j : 0u;                      // clamped, branch-free prefetch
        off = A.off[jc];
        len = j < lim ? (uint32_t)A.len[jc] : 0u;
    };
    uint64_t dn_o, dnn_o;
    uint32_t dn_l, dnn_l;
    uint32_t jA = piece_at(0u);
    desc(jA, dn_o, dn_l);
    desc(piece_at(1u), dnn_o, dnn_l);                              // two ahead
    uint32_t touch = 0u;
    if constexpr (TOUCH) {
        uint64_t to;
        uint32_t tl;
        const uint32_t ti = (uint32_t)lane >> 1, tb = ((uint32_t)lane & 1u) << 10;
        desc(ti < 4u && ti < iters ? piece_at(ti) : ~0u, to, tl);
        const uintptr_t ta = tb < tl ? base + to + tb : zero_addr();
        touch = *reinterpret_cast<const __attribute__((address_space(1))) uint32_t*>(ta);
    }
    PieceStage SA, SB;
    piece_issue(SA, base + dn_o, dn_l, lane);
    dn_o = dnn_o;
    dn_l = dnn_l;
    uint32_t b, h;
    for (uint32_t i = 0u; i < iters; i += 2u) {
        const uint32_t jB = piece_at(i + 1u);
        desc(piece_at(i + 2u), dnn_o, dnn_l);
        piece_issue(SB, base + dn_o, dn_l, lane);
        dn_o = dnn_o;
        dn_l = dnn_l;
        piece_consume(SA, lane, b, h);
        piece_store(eo, jA, b, h, lane, jA < lim);
        jA = piece_at(i + 2u);
        desc(piece_at(i + 3u), dnn_o, dnn_l);
        piece_issue(SA, base + dn_o, dn_l, lane);
        dn_o = dnn_o;
        dn_l = dnn_l;
        piece_consume(SB, lane, b, h);
        piece_store(eo, jB, b, h, lane, jB < lim);
    }
    asm volatile("" ::"v"(touch));                                 // (the touch is never used)
}

// Pass 1 in the live-sector stream (NETCSUM_TUNE_KERNEL 3; round 5): a wave takes a run of `spw` pieces
// and, when they lie in address order within 63 KiB of the run's first 128-B line (a datagram's
// fragments in their NET_BUFs, one per 2-KiB buffer at +42), reads only the 64-B sectors that hold
// piece bytes, as seg_live_varlen_kernel (netcsum_stream.hip) does for segments: a per-wave LDS
// bitmap of live sectors, the live 1-KiB pieces popped in address order, a lane loading its 16 B only
// where its sector is live. Each piece end is one scalar event taking two wave totals, the byte sum b
// and the half-word sum h of [start, end), into the piece's lane; a vector epilogue writes the records
// (e | o << 32, o = (h - b) / 255). Runs out of order or past the reach take pass 1's 16-lane groups.
// Measured on the chain row (16 Ki x 45 fragments): 0.1993-0.2046 ms in runs of 16-24 against
// 0.1756-0.1803 ms for the tiled groups (profiles/r5v_chains.log) — two wave totals per piece end
// cost more than the skipped sectors save — so the groups stay the default; the live-sector read
// floor of the fragments is 0.1550 ms (tools/live_read_probe.hip frag2k, profiles/r5k_*).
__device__ __forceinline__ uint32_t sum4b(u32x4 v) {
    uint32_t b = __builtin_amdgcn_sad_u8(v.x, 0u, 0u);
    b = __builtin_amdgcn_sad_u8(v.y, 0u, b);
    b = __builtin_amdgcn_sad_u8(v.z, 0u, b);
    return __builtin_amdgcn_sad_u8(v.w, 0u, b);
}
// piece_prefix (netcsum_stream.h) of the byte sum
__device__ __forceinline__ uint32_t piece_prefix_b(u32x4 v, uint32_t s4, uint32_t lane16, uint32_t x) {
    const uint32_t k = x & 15u;
    const uint64_t m0 = k >= 8u ? ~0ull : (1ull << (8u * k)) - 1ull;
    const uint64_t m1 = k <= 8u ? 0ull : (1ull << (8u * (k - 8u))) - 1ull;
    uint32_t pv = __builtin_amdgcn_sad_u8(v.x & (uint32_t)m0, 0u, 0u);
    pv = __builtin_amdgcn_sad_u8(v.y & (uint32_t)(m0 >> 32), 0u, pv);
    pv = __builtin_amdgcn_sad_u8(v.z & (uint32_t)m1, 0u, pv);
    pv = __builtin_amdgcn_sad_u8(v.w & (uint32_t)(m1 >> 32), 0u, pv);
    return (lane16 + 16u <= x) ? s4 : ((lane16 < x) ? pv : 0u);
}

template <int D>
__global__ void __launch_bounds__(256) chain_live_piece_kernel(ChainBatchArgs A, uint64_t* eo, uint32_t cap, uint32_t spw) {
    using namespace sv;
    __shared__ uint32_t sect_all[4][32];
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t np = *reinterpret_cast<c_u32*>(reinterpret_cast<uintptr_t>(A.first + A.n));
    if (np > cap) {                                               // no room for the records: the
        return;                                                   // combine pass does the batch
    }
    const uint64_t sb64 = ((uint64_t)blockIdx.x * 4u + w) * spw;
    if (sb64 >= np) {
        return;
    }
    const uint32_t s_begin = (uint32_t)sb64;
    const uint32_t nres = min(np - s_begin, spw);                 // spw <= 64: piece k in lane k
    const uint32_t lane16 = 16u * lane;
    const uintptr_t base = (uintptr_t)A.base;
    const bool mine = lane < nres;
    const uint64_t off = A.off[s_begin + (mine ? lane : 0u)];
    const uint32_t len = mine ? (uint32_t)A.len[s_begin + lane] : 0u;
    const uint64_t off0 = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(off >> 32)) << 32) |
                          (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)off);
    const uintptr_t O = (base + off0) & ~(uintptr_t)127;
    const uint64_t rel = base + off - O;
    const uint64_t end = rel + len;
    const uint32_t prev_end = (uint32_t)__shfl_up((int)(uint32_t)end, 1, 64);
    const bool ok = !mine || (rel < kLiveReach && end <= kLiveReach - 128u && (lane == 0u || (uint64_t)prev_end <= rel));
    if (__builtin_amdgcn_ballot_w64(!ok) != 0u) {
        // out of order, overlapping or past the reach: pass 1's 16-lane groups, four pieces at a time
        const int gl = (int)(lane & 15u);
        for (uint32_t k0 = 0; k0 < nres; k0 += 4u) {
            const uint32_t k = k0 + (lane >> 4);
            const uint64_t o = __shfl(off, (int)(k & 63u), 64);
            const uint32_t l = (uint32_t)__shfl((int)len, (int)(k & 63u), 64);
            // one 16-B chunk per lane at a time (this path is rare; pass 1's six-chunk stages set the
            // kernel's VGPR count: 79 against 5x, 6 waves per SIMD against 8)
            const uintptr_t a = base + o;
            const uint32_t ln = k < nres ? l : 0u;
            const uint32_t lead = (uint32_t)(a & 15u), rend = lead + ln;
            const uint32_t nch = ln ? (rend + 15u) >> 4 : 0u;
            const uintptr_t q0 = a & ~(uintptr_t)15;
            uint32_t b = 0u, h = 0u;
            uint32_t steps = (nch + 15u) >> 4;
            steps = max(steps, (uint32_t)__shfl_xor((int)steps, 16, 64));
            steps = max(steps, (uint32_t)__shfl_xor((int)steps, 32, 64));
            for (uint32_t t = 0; t < steps; ++t) {
                const uint32_t c = 16u * t + (uint32_t)gl;
                u32x4 v = load16<true>(reinterpret_cast<gu32x4*>(c < nch ? q0 + 16u * (uintptr_t)c : zero_addr()));
                if (c < nch) {
                    v = edge_mask_rel(v, c, lead, rend);
                }
                b += sum4b(v);
                h = sum4(v, h);
            }
            piece_store(eo, s_begin + k, b, h, gl, k < nres);
        }
        return;
    }
    const uint32_t span = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)end, (int)(nres - 1u));
    const __amdgpu_buffer_rsrc_t rd = run_rsrc(O, (span + 15u) & ~15u);
    const u32x4 w0 = buf_load16<false>(rd, (mine && len != 0u) ? ((uint32_t)rel & ~15u) : kOOB);   // touch
    uint32_t* sect = sect_all[w];
    if (lane < 32u) {
        sect[lane] = 0u;
    }
    __builtin_amdgcn_wave_barrier();
    if (mine && len != 0u) {
        const uint32_t s0 = (uint32_t)rel >> 6, s1 = ((uint32_t)end - 1u) >> 6;
        for (uint32_t d = s0 >> 5; d <= (s1 >> 5); ++d) {
            const uint32_t lo = max(s0, d << 5) - (d << 5), hi = min(s1, (d << 5) + 31u) - (d << 5);
            atomicOr(&sect[d], (2u << hi) - (1u << lo));
        }
    }
    __builtin_amdgcn_wave_barrier();
    const uint32_t pm0 = reinterpret_cast<const uint16_t*>(sect)[lane];
    uint64_t lm0 = __builtin_amdgcn_ballot_w64(pm0 != 0u);
    const uint32_t nlive = (uint32_t)__builtin_popcountll(lm0);
    constexpr uint64_t kSent = 1ull << 63;
    lm0 |= kSent;
    const uint32_t lbit = 1u << (lane >> 2);
    auto pop = [&]() -> uint32_t {
        const uint32_t q = (uint32_t)__builtin_ctzll(lm0);
        lm0 = (lm0 & (lm0 - 1u)) | kSent;
        return q;
    };
    auto live_voff = [&](uint32_t q) -> uint32_t {
        const uint32_t sm = (uint32_t)__builtin_amdgcn_readlane((int)pm0, (int)q);
        return (sm & lbit) ? (q << 10) + lane16 : kOOB;
    };
    u32x4 dv[D];
    uint32_t qd[D];
#pragma unroll
    for (int j = 0; j < D; ++j) {
        qd[j] = pop();
        dv[j] = buf_load16<true>(rd, live_voff(qd[j]));
    }
    uint64_t srest = __builtin_amdgcn_ballot_w64(mine && len != 0u);
    const bool any = srest != 0u;
    uint32_t cur = any ? (uint32_t)__builtin_ctzll(srest) : 63u;
    srest &= srest - 1u;
    uint32_t cs = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)rel, (int)cur);
    uint32_t ce = any ? cs + (uint32_t)__builtin_amdgcn_readlane((int)len, (int)cur) : ~0u;
    uint32_t ah = 0u, ab = 0u, th = 0u, tb = 0u;
    auto consume = [&](uint32_t q, u32x4 v) {
        const uint32_t qb = q << 10;
        const uint32_t pend = qb + 1024u;
        const uint32_t fh = sum4(v, 0u), fb = sum4b(v);
        uint32_t u = cur, c = cs, e = ce, xh = ah, xb = ab, yh = th, yb = tb;
        uint64_t rs = srest;
        if (e > pend) {                                          // no piece ends in this 1 KiB
            const uint32_t x = min(c - qb, 1024u);
            xh += (c <= qb) ? fh : fh - piece_prefix(v, fh, lane16, x);
            xb += (c <= qb) ? fb : fb - piece_prefix_b(v, fb, lane16, x);
        } else {
            uint32_t Ph = (c <= qb) ? 0u : piece_prefix(v, fh, lane16, c - qb);
            uint32_t Pb = (c <= qb) ? 0u : piece_prefix_b(v, fb, lane16, c - qb);
#pragma clang loop vectorize(disable) unroll(disable)
            do {
                const uint32_t xe = e <= qb ? 0u : e - qb;
                const uint32_t Eh = piece_prefix(v, fh, lane16, xe), Eb = piece_prefix_b(v, fb, lane16, xe);
                const uint32_t Th = wave_total(xh + (Eh - Ph)), Tb = wave_total(xb + (Eb - Pb));
                yh = (lane == u) ? Th : yh;
                yb = (lane == u) ? Tb : yb;
                xh = 0u;
                xb = 0u;
                const bool more = rs != 0u;
                u = more ? (uint32_t)__builtin_ctzll(rs) : 63u;
                rs &= rs - 1u;
                const uint32_t pe = e;
                c = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)rel, (int)u);
                e = more ? c + (uint32_t)__builtin_amdgcn_readlane((int)len, (int)u) : ~0u;
                const uint32_t xc = c <= qb ? 0u : min(c - qb, 1024u);
                Ph = (c == pe) ? Eh : piece_prefix(v, fh, lane16, xc);
                Pb = (c == pe) ? Eb : piece_prefix_b(v, fb, lane16, xc);
            } while (e <= pend);
            xh = fh - Ph;
            xb = fb - Pb;
        }
        cur = u;
        srest = rs;
        cs = c;
        ce = e;
        ah = xh;
        ab = xb;
        th = yh;
        tb = yb;
    };
    const uint32_t rounds = (nlive + (uint32_t)D - 1u) / (uint32_t)D;
    for (uint32_t r = 0; r < rounds; ++r) {
#pragma unroll
        for (int j = 0; j < D; ++j) {
            consume(qd[j], opaque_tuple(dv[j]));
            qd[j] = pop();
            dv[j] = buf_load16<true>(rd, live_voff(qd[j]));
            asm volatile("" ::: "memory");
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("" ::"v"(w0));
    if (mine) {                                                   // h - b = 255 o exactly (< 64 KiB)
        const uint32_t o = (th - tb) * 0xFEFEFEFFu;
        eo[s_begin + lane] = (uint64_t)(tb - o) | ((uint64_t)o << 32);
    }
}

// A 16-lane group per chain (4 chains per wave, independent loads in flight for all four), 16
// pieces per step.
constexpr int kCG = 16;

__global__ void __launch_bounds__(256) chain_combine_kernel(ChainBatchArgs A, const uint64_t* eo, uint32_t cap) {
    const uint32_t np = *reinterpret_cast<c_u32*>(reinterpret_cast<uintptr_t>(A.first + A.n));
    if (np > cap) {                                               // pass 1 had no room for the records:
        const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // the batch in the
        for (uint32_t ch = blockIdx.x * 4u + w; ch < A.n; ch += gridDim.x * 4u) {   // wave-per-chain
            wave_chain(A, ch);                                    // form here (out of pass 1, whose
        }                                                         // registers it set: 116 VGPRs)
        return;
    }
    const int lane = (int)(threadIdx.x & (kCG - 1));
    const uint32_t sh = (threadIdx.x & 63u) & ~(uint32_t)(kCG - 1);          // the group's ballot bits
    const uint32_t below = (1u << lane) - 1u;
    const uint32_t ngr = gridDim.x * (256u / kCG);
    // wave-uniform trip count: the wave's 4 groups take chains c0 .. c0 + 3 of each round
    const uint32_t c0 = blockIdx.x * (256u / kCG) + (threadIdx.x & ~63u) / kCG;
    const uint32_t rounds = c0 < A.n ? (A.n - c0 + ngr - 1u) / ngr : 0u;
    for (uint32_t r = 0u; r < rounds; ++r) {
        const uint32_t ch = c0 + r * ngr + (threadIdx.x & 63u) / kCG;
        const bool live = ch < A.n;
        const uint32_t p0 = live ? A.first[ch] : 0u;
        const uint32_t p1 = live ? A.first[ch + 1u] : 0u;
        uint64_t E = 0u, O = 0u;
        uint32_t par = 0u;                                        // stream parity at the next piece
        if (live && A.pseudo && A.pseudo_len) {
            uint32_t plen = A.pseudo_len;
            if (p0 == p1 && (plen & 1u)) {
                plen -= 1u;                                       // NULL chain quirk
            }
            const uintptr_t pa = (uintptr_t)A.pseudo + (uint64_t)ch * A.pseudo_stride;
            const EO s = span_eo<kCG>(pa, plen, lane);
            if (pa & 1u) { E += s.o; O += s.e; } else { E += s.e; O += s.o; }
            par = A.pseudo_len & 1u;                              // pieces follow ALL pseudo bytes
        }
        const uint32_t npc = p1 - p0;
        uint32_t steps = (npc + kCG - 1u) / kCG;
#pragma unroll
        for (int m = 32; m >= kCG; m >>= 1) {                     // the wave's longest chain
            steps = max(steps, (uint32_t)__shfl_xor((int)steps, m, 64));
        }
        for (uint32_t t = 0u; t < steps; ++t) {
            const uint32_t j = p0 + t * kCG + (uint32_t)lane;
            const bool v = j < p1;
            const uint32_t len = v ? (uint32_t)A.len[j] : 0u;
            const uint64_t off = v ? A.off[j] : 0u;
            const uint64_t rec = v ? eo[j] : 0u;
            const uint32_t odd = (uint32_t)(__ballot((len & 1u) != 0u) >> sh) & 0xFFFFu;
            const uint32_t spar = par ^ ((uint32_t)__popc(odd & below) & 1u);
            const uint32_t swap = ((uint32_t)((uintptr_t)A.base + off) & 1u) ^ spar;
            const uint32_t e = (uint32_t)rec, o = (uint32_t)(rec >> 32);
            E += swap ? o : e;
            O += swap ? e : o;
            par ^= (uint32_t)__popc(odd) & 1u;
        }
        E = group_sum64<kCG>(E);
        O = group_sum64<kCG>(O);
        if (live && lane == 0) {
            chain_out(A, ch, E, O);
        }
    }
}

// ---- one record per piece (round 6) ------------------------------------------------------------
// Pass 1 in the live-sector segment stream (launch_chain_live_records) leaves ONE number per piece: its
// exact half-word sum h = e + 256 o in the absolute LE frame (e / o: its bytes at even / odd
// addresses). A piece's share of the chain's big-endian word sum T is 256 e + o where its stream
// parity equals its address parity and e + 256 o = h where it differs, and 256 e + o ≡ 256 h (mod
// 65535). While T < 2^32 the reference's u32 accumulator never wraps (net_util.c:1554, :1685) and its
// fold is T's one's-complement residue — the value in [1, 0xFFFF] congruent to T mod 65535, 0 only for
// T = 0 — which is the fold of ANY non-negative S ≡ T (mod 65535) that is 0 exactly when T is: here
// S = Σ (swap ? h : 256 h) + 256 E_p + O_p of the pseudo-header, each term 0 only when its bytes are.
// T <= ceil(L / 2) x 0xFFFF < 2^32 for a chain of L <= 131 072 stream bytes (every IPv4 datagram,
// every IPv6 one short of a jumbogram); a longer chain, whose accumulator may wrap, is re-read by its
// group in the exact even / odd form (span_eo, as chain_batch_kernel) — correct, slower.
constexpr uint64_t kChainModMax = 131072u;

__device__ __forceinline__ uint32_t fold64(uint64_t s) {
    while (s >> 16) {
        s = (s & 0xFFFFu) + (s >> 16);
    }
    return (uint32_t)s;
}

// A CG-lane group per chain (CG 16: 4 chains per wave, 16 pieces per step; CG 64: a wave per chain,
// 64 pieces per step — a 45-fragment datagram in one step, one dependent memory round trip after the
// chain's bounds).
template <int CG>
__global__ void __launch_bounds__(256) chain_combine_h_kernel(ChainBatchArgs A, const uint32_t* hr, uint32_t cap) {
    const uint32_t np = *reinterpret_cast<c_u32*>(reinterpret_cast<uintptr_t>(A.first + A.n));
    if (np > cap) {                                               // pass 1 had no room for the records:
        const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // the wave-per-chain form
        for (uint32_t ch = blockIdx.x * 4u + w; ch < A.n; ch += gridDim.x * 4u) {
            wave_chain(A, ch);
        }
        return;
    }
    const int lane = (int)(threadIdx.x & (CG - 1));
    const uint32_t sh = (threadIdx.x & 63u) & ~(uint32_t)(CG - 1);          // the group's ballot bits
    const uint64_t gmask = CG == 64 ? ~0ull : ((1ull << CG) - 1u);
    const uint64_t below = (1ull << lane) - 1u;
    const uint32_t ngr = gridDim.x * (256u / CG);
    const uint32_t c0 = blockIdx.x * (256u / CG) + (threadIdx.x & ~63u) / CG;
    const uint32_t rounds = c0 < A.n ? (A.n - c0 + ngr - 1u) / ngr : 0u;
    const uintptr_t base = (uintptr_t)A.base;
    for (uint32_t r = 0u; r < rounds; ++r) {
        const uint32_t ch = c0 + r * ngr + (threadIdx.x & 63u) / CG;
        const bool live = ch < A.n;
        const uint32_t p0 = live ? A.first[ch] : 0u;
        const uint32_t p1 = live ? A.first[ch + 1u] : 0u;
        uint64_t S = 0u, L = 0u;                                  // this lane's share of S, of the lengths
        uint32_t plen = 0u, par = 0u;                             // par: stream parity at the next piece
        uintptr_t pa = 0u;
        if (live && A.pseudo && A.pseudo_len) {
            plen = A.pseudo_len;
            if (p0 == p1 && (plen & 1u)) {
                plen -= 1u;                                       // NULL chain quirk
            }
            pa = (uintptr_t)A.pseudo + (uint64_t)ch * A.pseudo_stride;
            const EO s = span_eo<CG>(pa, plen, lane);
            S += (pa & 1u) ? ((uint64_t)s.o << 8) + s.e : ((uint64_t)s.e << 8) + s.o;
            par = A.pseudo_len & 1u;                              // pieces follow ALL pseudo bytes
        }
        const uint32_t par0 = par;
        uint32_t steps = (p1 - p0 + CG - 1u) / CG;
#pragma unroll
        for (int m = 32; m >= CG; m >>= 1) {                      // the wave's longest chain
            steps = max(steps, (uint32_t)__shfl_xor((int)steps, m, 64));
        }
        // U steps' descriptors and records loaded before any is used: one memory round trip for a
        // chain of up to U x CG pieces after its bounds (a 45-fragment datagram: one)
        constexpr uint32_t U = 4u;
        for (uint32_t t0 = 0u; t0 < steps; t0 += U) {
            uint32_t len[U];
            uint64_t off[U], h[U];
#pragma unroll
            for (uint32_t u = 0; u < U; ++u) {
                const uint32_t j = p0 + (t0 + u) * CG + (uint32_t)lane;
                const bool v = t0 + u < steps && j < p1;
                len[u] = v ? (uint32_t)A.len[j] : 0u;
                off[u] = v ? A.off[j] : 0u;
                h[u] = v ? hr[j] : 0u;
            }
#pragma unroll
            for (uint32_t u = 0; u < U; ++u) {
                const uint64_t odd = (__ballot((len[u] & 1u) != 0u) >> sh) & gmask;
                const uint32_t spar = par ^ ((uint32_t)__popcll(odd & below) & 1u);
                const uint32_t swap = ((uint32_t)(base + off[u]) & 1u) ^ spar;
                S += swap ? h[u] : h[u] << 8;
                L += len[u];
                par ^= (uint32_t)__popcll(odd) & 1u;
            }
        }
        S = group_sum64<CG>(S);
        L = group_sum64<CG>(L);
        const bool big = live && L + plen > kChainModMax;         // group-uniform
        if (big) {                                                // the exact form (u32 wrap included)
            uint64_t E = 0u, O = 0u;
            if (plen != 0u) {
                const EO s = span_eo<CG>(pa, plen, lane);
                if (pa & 1u) { E += s.o; O += s.e; } else { E += s.e; O += s.o; }
            }
            uint32_t spos = par0;
            for (uint32_t j = p0; j < p1; ++j) {
                const uintptr_t a = base + A.off[j];
                const uint32_t len = A.len[j];
                const EO s = span_eo<CG>(a, len, lane);
                if (((uint32_t)(a & 1u)) != spos) { E += s.o; O += s.e; } else { E += s.e; O += s.o; }
                spos ^= (len & 1u);
            }
            E = group_sum64<CG>(E);
            O = group_sum64<CG>(O);
            if (lane == 0) {
                chain_out(A, ch, E, O);
            }
        } else if (live && lane == 0) {
            const uint32_t sum = fold64(S);
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

hipError_t launch_chain_two_pass_h(const ChainBatchArgs& a, uint32_t* rec, uint32_t cap, int cus, hipStream_t s,
                                   uint32_t spw, int depth, bool cmp, int combine_lanes) {
    hipError_t e = launch_chain_live_records(a, rec, cap, depth, spw, cmp, s);
    if (e != hipSuccess) return e;
    const uint32_t cg = combine_lanes == 64 ? 64u : 16u;
    const uint64_t blocks = ((uint64_t)a.n + 256u / cg - 1u) / (256u / cg);
    const unsigned g2 = (unsigned)std::min<uint64_t>(blocks, (uint64_t)std::max(cus, 1) * 64u);
    if (cg == 64u) {
        hipLaunchKernelGGL(chain_combine_h_kernel<64>, dim3(g2), dim3(256), 0, s, a, (const uint32_t*)rec, cap);
    } else {
        hipLaunchKernelGGL(chain_combine_h_kernel<16>, dim3(g2), dim3(256), 0, s, a, (const uint32_t*)rec, cap);
    }
    return hipGetLastError();
}

namespace {
thread_local TuneKnob g_chain_grid{-1};                          // NETCSUM_TUNE_CHAIN_GRID
}
void set_chain_grid(int v) {
    g_chain_grid.store(v);
}
int chain_grid() {
    const int v = g_chain_grid.load();
    return v < 0 ? 0 : v;
}

hipError_t launch_chain_two_pass(const ChainBatchArgs& a, uint64_t* eo, uint32_t cap, int cus, hipStream_t s, uint32_t live_spw,
                                 int live_depth) {
    if (live_spw != 0u) {                                          // pass 1 in the live-sector stream:
        const uint64_t waves = ((uint64_t)cap + live_spw - 1u) / live_spw;   // a wave per run of the most
        const dim3 g1((unsigned)((waves + 3u) / 4u));              // pieces the records hold; runs past
        if (live_depth == 4) {                                     // the batch's return at once
            hipLaunchKernelGGL(chain_live_piece_kernel<4>, g1, dim3(256), 0, s, a, eo, cap, live_spw);
        } else {
            hipLaunchKernelGGL(chain_live_piece_kernel<8>, g1, dim3(256), 0, s, a, eo, cap, live_spw);
        }
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        const uint64_t blocks = ((uint64_t)a.n + 15u) / 16u;
        const unsigned g2 = (unsigned)std::min<uint64_t>(blocks, (uint64_t)std::max(cus, 1) * 64u);
        hipLaunchKernelGGL(chain_combine_kernel, dim3(g2), dim3(256), 0, s, a, (const uint64_t*)eo, cap);
        return hipGetLastError();
    }
    // pass 1: blocks take tiles of 64 consecutive pieces round-robin (the piece count lives on the
    // device; blocks past the last tile return). Grid: 2 blocks per chain, at least the resident
    // blocks, at most one per tile the scratch holds — so a batch of up to 32 pieces per chain gets
    // one block per tile, which the dispatcher hands out as blocks finish: 16 Ki x 45 fragments
    // 0.1857 -> 0.1807 ms against the resident-sized grid, 21 248 empty blocks included
    // (profiles/r3w_chain_grid_ab.log, tools/r3w_cmd.sh). Pass 2: a 16-lane group per chain.
    static const int per_cu = [] {                                // thread-safe one-time query
        int nb = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, chain_piece_kernel<false, false>, 256, 0) != hipSuccess || nb <= 0) nb = 4;
        return nb;
    }();
    const uint64_t resident = (uint64_t)std::max(cus, 1) * (uint64_t)per_cu;
    // (at most 2^20 blocks = 2^28 threads, within the launch limit; the tiles go round-robin beyond)
    const uint64_t g1 = std::min<uint64_t>(std::min<uint64_t>(((uint64_t)cap + 63u) / 64u, 1ull << 20),
                                           std::max<uint64_t>(resident, 2ull * a.n));
    ChainBatchArgs ax = a;
    ax.xcd = stream_xcd_mode(1);
    const int cg = chain_grid();
    if (cg >= 1) {                                                 // balanced: cg x the resident blocks
        ax.xcd = stream_xcd(false) ? 1u : 0u;
        hipLaunchKernelGGL((chain_piece_kernel<true, false>), dim3((unsigned)(resident * (uint64_t)cg)), dim3(256), 0, s, ax,
                           eo, cap);
    } else if (stream_touch(false)) {
        hipLaunchKernelGGL((chain_piece_kernel<false, true>), dim3((unsigned)std::max<uint64_t>(g1, 1u)), dim3(256), 0, s, ax,
                           eo, cap);
    } else {
        hipLaunchKernelGGL((chain_piece_kernel<false, false>), dim3((unsigned)std::max<uint64_t>(g1, 1u)), dim3(256), 0, s, ax,
                           eo, cap);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const uint64_t blocks = ((uint64_t)a.n + 15u) / 16u;
    const unsigned g2 = (unsigned)std::min<uint64_t>(blocks, (uint64_t)std::max(cus, 1) * 64u);
    hipLaunchKernelGGL(chain_combine_kernel, dim3(g2), dim3(256), 0, s, a, (const uint64_t*)eo, cap);
    return hipGetLastError();
}

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
