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
#include <stdio.h>

#include "netcsum_device.h"
#include "netcsum_kernels.h"

namespace netcsum {

// Segment -> group mapping. Tile mode (P.tile = J > 0): block b owns the contiguous tile
// [b*gpb*J, (b+1)*gpb*J) and its gpb groups step through it gpb segments at a time, so the blocks
// in flight (dispatched in order) read one contiguous, advancing window of HBM. Grid-stride mode
// (P.tile = 0): group i handles i, i + G_total, ... (persistent grids).
struct SegRange {
    uint32_t first;
    uint32_t step;
    uint32_t end;
};

__device__ __forceinline__ SegRange seg_range(const SegBatchArgs& P, uint32_t gpb, uint32_t grp) {
    SegRange r;
    if (P.tile) {
        const uint64_t t0 = (uint64_t)blockIdx.x * gpb * P.tile;
        const uint64_t t1 = t0 + (uint64_t)gpb * P.tile;
        r.first = (uint32_t)(t0 + grp);
        r.step = gpb;
        r.end = (uint32_t)(t1 < P.n_seg ? t1 : P.n_seg);
    } else {
        r.first = blockIdx.x * gpb + grp;
        r.step = gridDim.x * gpb;
        r.end = P.n_seg;
    }
    return r;
}

// ---------------------------------------------------------------------------------------------
// Segment batch kernel. out[i] per NETCSUM_OP (include/netcsum_mi355x.h (2)).
// ---------------------------------------------------------------------------------------------
template <int G, int K, bool VARLEN, bool NT>
__global__ void __launch_bounds__(256) seg_batch_kernel(SegBatchArgs P) {
    const int      lane   = (int)(threadIdx.x & (G - 1));
    const uint32_t gpb    = blockDim.x / G;
    const bool     has_ph = (P.pseudo != nullptr) && (P.pseudo_len != 0u);
    const bool     ph_odd = (P.pseudo_len & 1u) != 0u;

    const SegRange R = seg_range(P, gpb, threadIdx.x / G);
    for (uint32_t seg = R.first; seg < R.end; seg += R.step) {
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
// v2: software-pipelined segment batch kernel.
//
// Each group keeps TWO segments in flight: while it masks, sums, folds and stores segment i, the
// K chunk loads (+ its pseudo-header chunk) of segment i+step are already issued. All loads are
// unconditional — a chunk slot past the end of its span reads a 16-byte zero chunk that lives in
// this code object (always mapped, L1/L2 resident) — so every load sits in straight-line code and
// the compiler's counted s_waitcnt vmcnt(N) waits only for the stage being consumed. For
// variable-length batches the (offset, length) descriptors are prefetched two segments ahead and
// issued BEFORE the data loads they gate, so waiting for a descriptor never drains the data
// stream (vmcnt retires in issue order).
// ---------------------------------------------------------------------------------------------
template <int K>
struct SegStage {
    u32x4    v[K];
    u32x4    pv;
    uint32_t lead;      // segment start offset inside its first 16-B chunk (bit 0 = address parity)
    uint32_t len;
    uint32_t plead;     // same for the pseudo-header
    uint32_t plen;      // pseudo-header bytes of THIS stage (0 for a dummy / past-the-end stage)
};

template <int G, int K, bool NT>
__device__ __forceinline__ void stage_issue(SegStage<K>& st, uintptr_t a, uint32_t len, uintptr_t pa,
                                            uint32_t plen, int lane) {
    st.lead = (uint32_t)(a & 15u);
    st.len = len;
    st.plead = (uint32_t)(pa & 15u);
    st.plen = plen;
    const uintptr_t q0 = a & ~(uintptr_t)15;
    const uint32_t nch = (len + st.lead + 15u) >> 4;            // 0 when len == 0 (lead < 16)
    const uintptr_t z = zero_addr();
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint32_t c = (uint32_t)(k * G + lane);
        const uintptr_t addr = (c < nch) ? (q0 + 16u * (uintptr_t)c) : z;
        st.v[k] = load16<NT>(reinterpret_cast<gu32x4*>(addr));
    }
    const uint32_t pnch = (plen + st.plead + 15u) >> 4;
    const uintptr_t paddr = ((uint32_t)lane < pnch) ? ((pa & ~(uintptr_t)15) + 16u * (uintptr_t)lane) : z;
    st.pv = load16<false>(reinterpret_cast<gu32x4*>(paddr));
}

// Folded 16-bit contribution of (pseudo ‖ segment) held by this lane, stream parity applied.
// `a`/`pa` (full addresses) are only needed for passes beyond the pipelined first one.
// Every address touched here derives from the STAGE's own (len, plen): a dummy stage (len = plen = 0)
// reads nothing beyond its zero-chunk slots.
template <int G, int K, bool NT>
__device__ __forceinline__ uint32_t stage_consume(const SegStage<K>& st, uintptr_t a, uintptr_t pa,
                                                  bool ph_odd, int lane) {
    const uint32_t plen = st.plen;
    const uint32_t lead = st.lead;
    const uint32_t rend = lead + st.len;
    const uint32_t nch = (rend + 15u) >> 4;
    uint32_t acc = 0u;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint32_t c = (uint32_t)(k * G + lane);
        u32x4 v = opaque(st.v[k]);
        if (c < nch) {
            v = edge_mask_rel(v, c, lead, rend);
        }
        acc = sum4(v, acc);
    }
    const u32x4 pv = opaque(st.pv);
    if (nch > (uint32_t)(G * K)) {                   // segments longer than one pass
        const uintptr_t q0 = a & ~(uintptr_t)15;
        for (uint32_t c0 = (uint32_t)(G * K); c0 < nch; c0 += (uint32_t)(G * K)) {
            u32x4 w[K];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const uint32_t c = c0 + (uint32_t)(k * G + lane);
                const uintptr_t addr = (c < nch) ? (q0 + 16u * (uintptr_t)c) : zero_addr();
                w[k] = load16<NT>(reinterpret_cast<gu32x4*>(addr));
            }
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const uint32_t c = c0 + (uint32_t)(k * G + lane);
                u32x4 v = w[k];
                if (c < nch) {
                    v = edge_mask_rel(v, c, lead, rend);
                }
                acc = sum4(v, acc);
            }
        }
    }
    uint32_t s = fold16(acc);
    if (((lead & 1u) != 0u) != ph_odd) {
        s = rot8(s);
    }
    if (plen != 0u) {
        const uint32_t plead = st.plead;
        const uint32_t prend = plead + plen;
        const uint32_t pnch = (prend + 15u) >> 4;
        u32x4 v = pv;
        if ((uint32_t)lane < pnch) {
            v = edge_mask_rel(v, (uint32_t)lane, plead, prend);
        }
        uint32_t pacc = sum4(v, 0u);
        if (pnch > (uint32_t)G) {                    // pseudo-header longer than 16*G - 15 B
            const uintptr_t pq0 = pa & ~(uintptr_t)15;
            for (uint32_t c = (uint32_t)(lane + G); c < pnch; c += (uint32_t)G) {
                const u32x4 w = load16<false>(reinterpret_cast<gu32x4*>(pq0 + 16u * (uintptr_t)c));
                pacc = sum4(edge_mask_rel(w, c, plead, prend), pacc);
            }
        }
        uint32_t ps = fold16(pacc);
        if (plead & 1u) {
            ps = rot8(ps);
        }
        s += ps;
    }
    return s;
}

template <int G>
__device__ __forceinline__ void group_store(const SegBatchArgs& P, uint32_t seg, uint32_t s, int lane) {
    s = fold16(group_sum<G>(s));
    if (lane == 0) {
        if (P.verify) {
            static_cast<uint8_t*>(P.out)[seg] = (s == 0xFFFFu) ? 1u : 0u;
        } else {
            static_cast<uint16_t*>(P.out)[seg] = (uint16_t)(~s);
        }
    }
}

template <bool VARLEN>
struct SegDesc {
    uint64_t off;
    uint32_t len;
};

template <bool VARLEN>
__device__ __forceinline__ SegDesc<VARLEN> seg_desc(const SegBatchArgs& P, uint32_t seg) {
    SegDesc<VARLEN> d;
    if constexpr (VARLEN) {
        const uint32_t sc = (seg < P.n_seg) ? seg : 0u;          // clamped, branch-free prefetch
        d.off = P.seg_off[sc];
        d.len = P.seg_len_v[sc];
    } else {
        d.off = (uint64_t)seg * P.seg_stride;
        d.len = P.seg_len;
    }
    return d;
}

template <int G, int K, bool VARLEN, bool NT>
__global__ void __launch_bounds__(256) seg_pipe_kernel(SegBatchArgs P) {
    const int      lane = (int)(threadIdx.x & (G - 1));
    const uint32_t gpb  = blockDim.x / G;
    const uint32_t plen = (P.pseudo != nullptr) ? P.pseudo_len : 0u;
    const bool     ph_odd = (plen & 1u) != 0u;
    const uintptr_t base = (uintptr_t)P.base;
    const uintptr_t pbase = (uintptr_t)P.pseudo;
    const uintptr_t z = zero_addr();

    const SegRange R = seg_range(P, gpb, threadIdx.x / G);
    const uint32_t step = R.step;
    const uint32_t cnt = group_iters(R.first, step, R.end);
    const uint32_t iters = __builtin_amdgcn_readfirstlane(cnt);
    if (iters == 0u) {
        return;
    }
    uint32_t seg = R.first;
    SegStage<K> A, B;
    SegDesc<VARLEN> dn = seg_desc<VARLEN>(P, seg);
    SegDesc<VARLEN> dnn = seg_desc<VARLEN>(P, seg + step);      // two ahead
    bool vA = cnt != 0u, vB = false;
    uintptr_t aA = vA ? base + dn.off : z, paA = vA ? pbase + (uint64_t)seg * P.pseudo_stride : z;
    uintptr_t aB = z, paB = z;
    stage_issue<G, K, NT>(A, aA, vA ? dn.len : 0u, paA, vA ? plen : 0u, lane);
    dn = dnn;
    // Wave-uniform trip count (group_iters) and ONE exit, at the latch: a group past its own end
    // runs dummy stages (zero-chunk loads) and stores nothing. (A mid-body `break`, even a
    // uniform one, leaves the structurizer's never-taken edge from the first half back to the
    // header, on which stage B is still pending — and the waitcnt pass drains vmcnt(0) for it.)
    for (uint32_t j = 0u; j < iters; j += 2u) {
        // ---- consume A (iteration j) with B (j + 1) in flight
        uint32_t nxt = seg + step;
        vB = j + 1u < cnt;
        dnn = seg_desc<VARLEN>(P, nxt + step);
        aB = vB ? base + dn.off : z;
        paB = vB ? pbase + (uint64_t)nxt * P.pseudo_stride : z;
        stage_issue<G, K, NT>(B, aB, vB ? dn.len : 0u, paB, vB ? plen : 0u, lane);
        dn = dnn;
        uint32_t r = stage_consume<G, K, NT>(A, aA, paA, ph_odd, lane);
        if (vA) {                                             // uniform within the group
            group_store<G>(P, seg, r, lane);
        }
        seg = nxt;
        // ---- consume B (j + 1) with A (j + 2) in flight
        nxt = seg + step;
        vA = j + 2u < cnt;
        dnn = seg_desc<VARLEN>(P, nxt + step);
        aA = vA ? base + dn.off : z;
        paA = vA ? pbase + (uint64_t)nxt * P.pseudo_stride : z;
        stage_issue<G, K, NT>(A, aA, vA ? dn.len : 0u, paA, vA ? plen : 0u, lane);
        dn = dnn;
        r = stage_consume<G, K, NT>(B, aB, paB, ph_odd, lane);
        if (vB) {
            group_store<G>(P, seg, r, lane);
        }
        seg = nxt;
    }
}

// ---------------------------------------------------------------------------------------------
// v3: the v2 pipeline with the segment stream moved onto LDS-DMA.
//
// Segment chunks are fetched by global_load_lds_dwordx4 (per-lane source address = the same
// clamped chunk addressing as v2; destination = this wave's slot in an LDS ring, lane i's 16 B at
// slot + 16*i) with the non-temporal policy, and read back by the same lane with ds_read_b128
// (conflict-free: 64 consecutive 16-B slots). On gfx950 this path streams HBM measurably faster
// than register-destination loads (bench: read_stream_lds probe vs read_stream probe). The
// pseudo-header chunk rides in slot K the same way, so no VGPR-destination load is ever in flight
// across an iteration (a pending VGPR load whose register the allocator re-uses forces a full
// vmcnt(0) drain). Nothing orders a ds_read behind an LDS-DMA except the issuing wave's vmcnt, so
// the waits are hand-counted: every stage issues exactly K+1 DMA, and consuming stage X while
// stage Y (issued after X) is in flight waits vmcnt(K+1) — conservative if anything else (stores,
// descriptor loads) was issued after Y.
// LDS: 2 stages x (K+1) slots x 1 KiB per wave.
// ---------------------------------------------------------------------------------------------
template <int K>
struct LdsStage {
    uint32_t lead;
    uint32_t len;
    uint32_t plead;
    uint32_t plen;
};

template <int G, int K, bool NT>
__device__ __forceinline__ void lds_stage_issue(LdsStage<K>& st, u32x4 (*slots)[64], uintptr_t a, uint32_t len,
                                                uintptr_t pa, uint32_t plen, int lane) {
    st.lead = (uint32_t)(a & 15u);
    st.len = len;
    st.plead = (uint32_t)(pa & 15u);
    st.plen = plen;
    const uintptr_t q0 = a & ~(uintptr_t)15;
    const uint32_t nch = (len + st.lead + 15u) >> 4;
    const uintptr_t z = zero_addr();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");        // prior ds_reads of these slots done
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint32_t c = (uint32_t)(k * G + lane);
        const uintptr_t addr = (c < nch) ? (q0 + 16u * (uintptr_t)c) : z;
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const __attribute__((address_space(1))) void*>(addr),
                                         (lds_void*)(&slots[k][0]), 16, 0, NT ? 2 : 0);
    }
    const uint32_t pnch = (plen + st.plead + 15u) >> 4;
    const uintptr_t paddr = ((uint32_t)lane < pnch) ? ((pa & ~(uintptr_t)15) + 16u * (uintptr_t)lane) : z;
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const __attribute__((address_space(1))) void*>(paddr),
                                     (lds_void*)(&slots[K][0]), 16, 0, 0);
}

template <int G, int K, bool NT>
__device__ __forceinline__ uint32_t lds_stage_consume(const LdsStage<K>& st, u32x4 (*slots)[64], uintptr_t a,
                                                      uintptr_t pa, bool ph_odd, int lane, int lane64) {
    SegStage<K> r;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        r.v[k] = slots[k][lane64];
    }
    r.pv = slots[K][lane64];
    r.lead = st.lead;
    r.len = st.len;
    r.plead = st.plead;
    r.plen = st.plen;
    return stage_consume<G, K, NT>(r, a, pa, ph_odd, lane);
}

template <int G, int K, bool VARLEN, bool NT>
__global__ void __launch_bounds__(256) seg_lds_kernel(SegBatchArgs P) {
    __shared__ u32x4 ring[4][2][K + 1][64];
    const int      w = (int)(threadIdx.x >> 6);
    const int      lane64 = (int)(threadIdx.x & 63);
    const int      lane = (int)(threadIdx.x & (G - 1));
    const uint32_t gpb  = blockDim.x / G;
    const uint32_t plen = (P.pseudo != nullptr) ? P.pseudo_len : 0u;
    const bool     ph_odd = (plen & 1u) != 0u;
    const uintptr_t base = (uintptr_t)P.base;
    const uintptr_t pbase = (uintptr_t)P.pseudo;
    const uintptr_t z = zero_addr();
    u32x4 (*sA)[64] = ring[w][0];
    u32x4 (*sB)[64] = ring[w][1];

    const SegRange R = seg_range(P, gpb, threadIdx.x / G);
    const uint32_t step = R.step;
    uint32_t seg = R.first;
    // Groups of one wave may run out of segments at different iterations; a finished group keeps
    // issuing zero-chunk stages (len 0) so every lane of the wave executes the same DMA sequence
    // and the hand-counted waits stay exact, and leaves only when the whole wave is done.
    const SegRange Rw = seg_range(P, gpb, (uint32_t)(w * 64) / G);
    if (Rw.first >= Rw.end) {
        return;
    }
    LdsStage<K> A, B;
    bool live = seg < R.end;
    SegDesc<VARLEN> dn = seg_desc<VARLEN>(P, seg);
    SegDesc<VARLEN> dnn = seg_desc<VARLEN>(P, seg + step);
    uintptr_t aA = live ? base + dn.off : z, paA = live ? pbase + (uint64_t)seg * P.pseudo_stride : z;
    uintptr_t aB = z, paB = z;
    lds_stage_issue<G, K, NT>(A, sA, aA, live ? dn.len : 0u, paA, live ? plen : 0u, lane);
    dn = dnn;
    for (;;) {
        uint32_t nxt = seg + step;
        bool has_next = nxt < R.end;
        dnn = seg_desc<VARLEN>(P, nxt + step);
        aB = has_next ? base + dn.off : z;
        paB = has_next ? pbase + (uint64_t)nxt * P.pseudo_stride : z;
        lds_stage_issue<G, K, NT>(B, sB, aB, has_next ? dn.len : 0u, paB, has_next ? plen : 0u, lane);
        dn = dnn;
        wait_vmcnt<K + 1>();
        {
            const uint32_t r = lds_stage_consume<G, K, NT>(A, sA, aA, paA, ph_odd, lane, lane64);
            if (live) {
                group_store<G>(P, seg, r, lane);
            }
        }
        live = has_next;
        if (!__any(has_next)) {
            break;
        }
        seg = nxt;
        nxt = seg + step;
        has_next = nxt < R.end;
        dnn = seg_desc<VARLEN>(P, nxt + step);
        aA = has_next ? base + dn.off : z;
        paA = has_next ? pbase + (uint64_t)nxt * P.pseudo_stride : z;
        lds_stage_issue<G, K, NT>(A, sA, aA, has_next ? dn.len : 0u, paA, has_next ? plen : 0u, lane);
        dn = dnn;
        wait_vmcnt<K + 1>();
        {
            const uint32_t r = lds_stage_consume<G, K, NT>(B, sB, aB, paB, ph_odd, lane, lane64);
            if (live) {
                group_store<G>(P, seg, r, lane);
            }
        }
        live = has_next;
        if (!__any(has_next)) {
            break;
        }
        seg = nxt;
    }
    wait_vmcnt<0>();                                           // drain the trailing stage's DMA
}

// ---------------------------------------------------------------------------------------------
// v4: wave-tile streaming through an LDS image (strided batches with stride >= length).
//
// A wave owns a TILE of S = 64/G consecutive segments. Their bytes — one contiguous range of
// HBM — are fetched as P whole 1-KiB LDS-DMA pieces starting at the 128-B line below the first
// segment, so every wave-instruction reads 8 full, aligned cache lines (the read-probe pattern)
// instead of G-lane pieces at 16-B alignment. The tile's pseudo-headers (contiguous too) ride in
// one extra piece. Each G-lane group then reads ITS segment's 16-B chunks back from the LDS
// image (aligned ds_read_b128), masks the edges and sums exactly as v2. Two stages per wave
// (ping-pong), hand-counted vmcnt(P+1). Host guarantees (S-1)*stride + len + 127 <= P*1024,
// K*G >= chunks per segment and (S-1)*pstride + plen + 15 <= 1024.
// ---------------------------------------------------------------------------------------------
struct TileStage {
    uint32_t seg0;       // first segment of the tile
    uint32_t nseg;       // segments of this tile (< S only for the last tile; 0 = dummy)
    uint32_t img_lead;   // tile start - image start (image start is 128-B aligned)
    uint32_t pimg_lead;  // pseudo-header range start - its 16-B aligned image start
};

template <int G, int P, bool NT>
__device__ __forceinline__ void tile_issue(TileStage& st, u32x4 (*img)[64], const SegBatchArgs& A, uint32_t tile,
                                           uint32_t ntiles, uint32_t plen, int lane64) {
    constexpr uint32_t S = 64 / G;
    const uintptr_t z = zero_addr();
    const bool live = tile < ntiles;
    st.seg0 = tile * S;
    st.nseg = live ? min(S, A.n_seg - st.seg0) : 0u;
    const uintptr_t a0 = (uintptr_t)A.base + (uint64_t)st.seg0 * A.seg_stride;
    // zero-length segments read nothing (the "buffer" may not exist at all)
    const uintptr_t aend = (live && A.seg_len) ? a0 + (uint64_t)(st.nseg - 1u) * A.seg_stride + A.seg_len : 0u;
    const uintptr_t img0 = a0 & ~(uintptr_t)127;
    st.img_lead = (uint32_t)(a0 - img0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");       // prior ds_reads of this stage done
#pragma unroll
    for (int p = 0; p < P; ++p) {
        const uintptr_t src = img0 + 1024u * (uintptr_t)p + 16u * (uintptr_t)lane64;
        __builtin_amdgcn_global_load_lds(
            reinterpret_cast<const __attribute__((address_space(1))) void*>(src < aend ? src : z),
            (lds_void*)(&img[p][0]), 16, 0, NT ? 2 : 0);
    }
    const uintptr_t p0 = (uintptr_t)A.pseudo + (uint64_t)st.seg0 * A.pseudo_stride;
    const uintptr_t pend = (live && plen) ? p0 + (uint64_t)(st.nseg - 1u) * A.pseudo_stride + plen : 0u;
    const uintptr_t pimg0 = p0 & ~(uintptr_t)15;
    st.pimg_lead = (uint32_t)(p0 - pimg0);
    const uintptr_t psrc = pimg0 + 16u * (uintptr_t)lane64;
    __builtin_amdgcn_global_load_lds(
        reinterpret_cast<const __attribute__((address_space(1))) void*>(psrc < pend ? psrc : z),
        (lds_void*)(&img[P][0]), 16, 0, 0);
}

template <int G, int P, int K>
__device__ __forceinline__ void tile_consume(const TileStage& st, u32x4 (*img)[64], const SegBatchArgs& A,
                                             uint32_t plen, bool ph_odd, int lane64) {
    const int g = lane64 / G;
    const int lane = lane64 & (G - 1);
    const u32x4* flat = &img[0][0];
    const uint32_t so = st.img_lead + (uint32_t)g * (uint32_t)A.seg_stride;   // < P*1024 (host check)
    const uint32_t lead = so & 15u;
    const uint32_t rend = lead + A.seg_len;
    const uint32_t nch = (rend + 15u) >> 4;
    const uint32_t cb = so >> 4;
    uint32_t acc = 0u;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint32_t c = (uint32_t)(k * G + lane);
        if (c < nch) {
            acc = sum4(edge_mask_rel(flat[cb + c], c, lead, rend), acc);
        }
    }
    uint32_t s = fold16(acc);
    if (((lead & 1u) != 0u) != ph_odd) {
        s = rot8(s);
    }
    if (plen != 0u) {
        const u32x4* pflat = &img[P][0];
        const uint32_t pso = st.pimg_lead + (uint32_t)g * A.pseudo_stride;   // < 1024 (host check)
        const uint32_t plead = pso & 15u;
        const uint32_t prend = plead + plen;
        const uint32_t pnch = (prend + 15u) >> 4;
        uint32_t pacc = 0u;
        for (uint32_t c = (uint32_t)lane; c < pnch; c += (uint32_t)G) {
            pacc = sum4(edge_mask_rel(pflat[(pso >> 4) + c], c, plead, prend), pacc);
        }
        uint32_t ps = fold16(pacc);
        if (plead & 1u) {
            ps = rot8(ps);
        }
        s += ps;
    }
    s = fold16(group_sum<G>(s));
    if (lane == 0 && (uint32_t)g < st.nseg) {
        const uint32_t seg = st.seg0 + (uint32_t)g;
        if (A.verify) {
            static_cast<uint8_t*>(A.out)[seg] = (s == 0xFFFFu) ? 1u : 0u;
        } else {
            static_cast<uint16_t*>(A.out)[seg] = (uint16_t)(~s);
        }
    }
}

template <int G, int P, int K, bool NT>
__global__ void __launch_bounds__(256) seg_tile_kernel(SegBatchArgs A) {
    constexpr uint32_t S = 64 / G;
    __shared__ u32x4 img[4][2][P + 1][64];
    const int w = (int)(threadIdx.x >> 6);
    const int lane64 = (int)(threadIdx.x & 63);
    const uint32_t plen = (A.pseudo != nullptr) ? A.pseudo_len : 0u;
    const bool ph_odd = (plen & 1u) != 0u;
    const uint32_t ntiles = (A.n_seg + S - 1u) / S;
    uint32_t t, tstep, tend;                                    // wave-uniform tile walk
    if (A.tile) {
        const uint64_t t0 = (uint64_t)blockIdx.x * 4u * A.tile;
        t = (uint32_t)t0 + (uint32_t)w;
        tstep = 4u;
        tend = (uint32_t)min<uint64_t>(t0 + 4ull * A.tile, ntiles);
    } else {
        t = blockIdx.x * 4u + (uint32_t)w;
        tstep = gridDim.x * 4u;
        tend = ntiles;
    }
    if (t >= tend) {
        return;
    }
    u32x4 (*sA)[64] = img[w][0];
    u32x4 (*sB)[64] = img[w][1];
    TileStage A0, B0;
    tile_issue<G, P, NT>(A0, sA, A, t, tend, plen, lane64);
    for (;;) {
        uint32_t nt = t + tstep;
        tile_issue<G, P, NT>(B0, sB, A, nt, tend, plen, lane64);   // dummy (reads zero chunk) past end
        wait_vmcnt<P + 1>();
        tile_consume<G, P, K>(A0, sA, A, plen, ph_odd, lane64);
        if (nt >= tend) {
            break;
        }
        t = nt;
        nt = t + tstep;
        tile_issue<G, P, NT>(A0, sA, A, nt, tend, plen, lane64);
        wait_vmcnt<P + 1>();
        tile_consume<G, P, K>(B0, sB, A, plen, ph_odd, lane64);
        if (nt >= tend) {
            break;
        }
        t = nt;
    }
    wait_vmcnt<0>();                                            // drain the trailing dummy stage
}

// ---------------------------------------------------------------------------------------------
// Roofline probe, LDS-DMA form: global_load_lds_dwordx4 pieces (1 KiB per wave-instruction)
// into a per-wave double-buffered LDS ring, counted vmcnt, ds_read_b128 + v_sad_u16 consumers.
// ---------------------------------------------------------------------------------------------
template <bool NT>
__global__ void __launch_bounds__(256) read_stream_lds_kernel(gu32x4* __restrict__ p, uint64_t n16,
                                                              unsigned long long* __restrict__ sink) {
    constexpr int P4 = 4;                                  // pieces per batch per wave
    __shared__ u32x4 ring[4][2][P4][64];
    const int w = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63);
    const uint64_t per_batch = (uint64_t)gridDim.x * 4u * P4 * 64u;   // chunks per grid-wide batch
    uint64_t c = ((uint64_t)blockIdx.x * 4u + (uint64_t)w) * (P4 * 64u) + (uint64_t)lane;
    const uint64_t nb = n16 / per_batch;                   // full batches only (probe)
    uint32_t acc = 0u;
    constexpr int aux = NT ? 2 : 0;
    auto issue = [&](uint64_t cc, int slot) {
#pragma unroll
        for (int j = 0; j < P4; ++j) {
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(p + cc + 64u * j),
                                             (__attribute__((address_space(3))) void*)&ring[w][slot][j][0], 16, 0, aux);
        }
    };
    if (nb > 0) {
        issue(c, 0);
    }
    for (uint64_t b = 0; b < nb; ++b) {
        const int slot = (int)(b & 1u);
        if (b + 1 < nb) {
            issue(c + per_batch, slot ^ 1);
            asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
#pragma unroll
        for (int j = 0; j < P4; ++j) {
            acc = sum4(ring[w][slot][j][lane], acc);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        c += per_batch;
    }
    // tail past the last whole batch: plain grid-stride loads, so the probe reads every byte
    const uint64_t tstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t t = nb * per_batch + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n16; t += tstride) {
        acc = sum4(load16<NT>(p + t), acc);
    }
    if (acc == 0x5EEDF00Du) {
        atomicAdd(sink, 1ull);
    }
}

// ---------------------------------------------------------------------------------------------
// Exact big-endian stream sum (host per-packet path): *sum += Σ BE 16-bit words of
// [p, p + n16*16). The stream is staged 16-byte aligned and zero padded by the host, so stream
// position == address and the pad adds nothing. v_perm_b32 swaps the bytes of both halves, then
// v_sad_u16 adds the two big-endian words: exact, no modular folding (the u32 wrap of the
// reference's cross-buffer `sum` is applied by the caller).
// ---------------------------------------------------------------------------------------------
// direct != 0 (single-block launches): thread 0 STORES the block total (no pre-zeroed accumulator
// needed — the per-packet path reads pinned host memory zero-copy and writes the result straight
// back into pinned host memory, one launch per call).
__global__ void __launch_bounds__(256) stream_exact_kernel(gu32x4* __restrict__ p, uint32_t n16,
                                                           unsigned long long* __restrict__ sum, int direct,
                                                           uint32_t tag) {
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
        if (direct && tag != 0u) {
            // completion word for a host that polls instead of synchronising: tag in the high half,
            // the reference's u32 sum in the low half, one system-scope release store
            __hip_atomic_store(sum, ((unsigned long long)tag << 32) | (uint32_t)t, __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        } else if (direct) {
            *sum = t;
        } else {
            atomicAdd(sum, t);
        }
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

// Persistent-grid sizing: blocks = (resident blocks per CU for this instantiation) x CUs x mult,
// so every workgroup is co-resident and they finish together (a partial last "round" of blocks
// leaves CUs idle for a whole block lifetime). Residency is cached per (instantiation, block).
template <typename Kern>
static int pick_grid(Kern kern, const LaunchCfg& c) {
    if (c.tile > 0) {                                    // one block per tile of gpb*tile segments
        const uint64_t per = (uint64_t)(c.block / c.group_lanes) * (uint64_t)c.tile;
        const uint64_t nseg = c.blocks_needed * (uint64_t)(c.block / c.group_lanes);
        return (int)((nseg + per - 1u) / per);
    }
    if (c.grid > 0) return c.grid;
    // residency per (kernel instantiation, block size), queried once
    struct OccEntry {
        const void* fn;
        int block;
        int occ;
    };
    static thread_local OccEntry cache[64];
    static thread_local int n_cache = 0;
    const void* fn = reinterpret_cast<const void*>(kern);
    int occ = 0;
    for (int i = 0; i < n_cache; ++i) {
        if (cache[i].fn == fn && cache[i].block == c.block) {
            occ = cache[i].occ;
            break;
        }
    }
    if (occ <= 0) {
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, c.block, 0) != hipSuccess || occ <= 0) {
            occ = 1;
        }
        if (n_cache < 64) {
            cache[n_cache++] = OccEntry{fn, c.block, occ};
        }
    }
    uint64_t g = (uint64_t)occ * (uint64_t)c.cus * (uint64_t)(c.grid_mult > 0 ? c.grid_mult : 1);
    if (g > c.blocks_needed) g = c.blocks_needed;
    return (int)(g ? g : 1);
}

template <int G, int K, bool VARLEN, bool NT>
static hipError_t launch_seg(const SegBatchArgs& a, const LaunchCfg& c, hipStream_t s) {
    const int grid = pick_grid(seg_batch_kernel<G, K, VARLEN, NT>, c);
    hipLaunchKernelGGL((seg_batch_kernel<G, K, VARLEN, NT>), dim3(grid), dim3(c.block), 0, s, a);
    return hipGetLastError();
}

template <int G, int K, bool VARLEN>
static hipError_t launch_seg_nt(const SegBatchArgs& a, const LaunchCfg& c, bool nt, hipStream_t s) {
    return nt ? launch_seg<G, K, VARLEN, true>(a, c, s)
              : launch_seg<G, K, VARLEN, false>(a, c, s);
}

template <int G, bool VARLEN>
static hipError_t launch_seg_k(const SegBatchArgs& a, int k, const LaunchCfg& c, bool nt, hipStream_t s) {
    switch (k) {
    case 1:  return launch_seg_nt<G, 1, VARLEN>(a, c, nt, s);
    case 2:  return launch_seg_nt<G, 2, VARLEN>(a, c, nt, s);
    case 3:  return launch_seg_nt<G, 3, VARLEN>(a, c, nt, s);
    default: return launch_seg_nt<G, 4, VARLEN>(a, c, nt, s);
    }
}

template <bool VARLEN>
static hipError_t launch_seg_g(const SegBatchArgs& a, int g, int k, const LaunchCfg& c, bool nt,
                               hipStream_t s) {
    switch (g) {
    case 1:  return launch_seg_k<1, VARLEN>(a, k, c, nt, s);
    case 4:  return launch_seg_k<4, VARLEN>(a, k, c, nt, s);
    case 8:  return launch_seg_k<8, VARLEN>(a, k, c, nt, s);
    case 16: return launch_seg_k<16, VARLEN>(a, k, c, nt, s);
    case 32: return launch_seg_k<32, VARLEN>(a, k, c, nt, s);
    default: return launch_seg_k<64, VARLEN>(a, k, c, nt, s);
    }
}

template <int G, int K, bool VARLEN, bool NT>
static hipError_t launch_pipe(const SegBatchArgs& a, const LaunchCfg& c, hipStream_t s) {
    const int grid = pick_grid(seg_pipe_kernel<G, K, VARLEN, NT>, c);
    hipLaunchKernelGGL((seg_pipe_kernel<G, K, VARLEN, NT>), dim3(grid), dim3(c.block), 0, s, a);
    return hipGetLastError();
}

template <int G, bool VARLEN, bool NT>
static hipError_t launch_pipe_k(const SegBatchArgs& a, int k, const LaunchCfg& c, hipStream_t s) {
    switch (k) {
    case 1:  return launch_pipe<G, 1, VARLEN, NT>(a, c, s);
    case 2:  return launch_pipe<G, 2, VARLEN, NT>(a, c, s);
    case 3:  return launch_pipe<G, 3, VARLEN, NT>(a, c, s);
    case 4:  return launch_pipe<G, 4, VARLEN, NT>(a, c, s);
    case 6:  return launch_pipe<G, 6, VARLEN, NT>(a, c, s);
    default: return launch_pipe<G, 8, VARLEN, NT>(a, c, s);
    }
}

template <bool VARLEN, bool NT>
static hipError_t launch_pipe_g(const SegBatchArgs& a, int g, int k, const LaunchCfg& c, hipStream_t s) {
    switch (g) {
    case 1:  return launch_pipe_k<1, VARLEN, NT>(a, k, c, s);
    case 4:  return launch_pipe_k<4, VARLEN, NT>(a, k, c, s);
    case 8:  return launch_pipe_k<8, VARLEN, NT>(a, k, c, s);
    case 16: return launch_pipe_k<16, VARLEN, NT>(a, k, c, s);
    case 32: return launch_pipe_k<32, VARLEN, NT>(a, k, c, s);
    default: return launch_pipe_k<64, VARLEN, NT>(a, k, c, s);
    }
}

template <int G, int K, bool VARLEN, bool NT>
static hipError_t launch_lds(const SegBatchArgs& a, const LaunchCfg& c, hipStream_t s) {
    const int grid = pick_grid(seg_lds_kernel<G, K, VARLEN, NT>, c);
    hipLaunchKernelGGL((seg_lds_kernel<G, K, VARLEN, NT>), dim3(grid), dim3(c.block), 0, s, a);
    return hipGetLastError();
}

template <int G, bool VARLEN, bool NT>
static hipError_t launch_lds_k(const SegBatchArgs& a, int k, const LaunchCfg& c, hipStream_t s) {
    switch (k) {
    case 1:  return launch_lds<G, 1, VARLEN, NT>(a, c, s);
    case 2:  return launch_lds<G, 2, VARLEN, NT>(a, c, s);
    case 3:  return launch_lds<G, 3, VARLEN, NT>(a, c, s);
    case 4:  return launch_lds<G, 4, VARLEN, NT>(a, c, s);
    case 6:  return launch_lds<G, 6, VARLEN, NT>(a, c, s);
    default: return launch_lds<G, 8, VARLEN, NT>(a, c, s);
    }
}

template <bool VARLEN, bool NT>
static hipError_t launch_lds_g(const SegBatchArgs& a, int g, int k, const LaunchCfg& c, hipStream_t s) {
    switch (g) {
    case 1:  return launch_lds_k<1, VARLEN, NT>(a, k, c, s);
    case 4:  return launch_lds_k<4, VARLEN, NT>(a, k, c, s);
    case 8:  return launch_lds_k<8, VARLEN, NT>(a, k, c, s);
    case 16: return launch_lds_k<16, VARLEN, NT>(a, k, c, s);
    case 32: return launch_lds_k<32, VARLEN, NT>(a, k, c, s);
    default: return launch_lds_k<64, VARLEN, NT>(a, k, c, s);
    }
}

template <int G, int P, int K, bool NT>
static hipError_t launch_tile(const SegBatchArgs& a, const LaunchCfg& c, hipStream_t s) {
    int grid;
    if (c.tile > 0) {
        const uint64_t tiles = ((uint64_t)a.n_seg + (64 / G) - 1u) / (64 / G);
        const uint64_t per = 4ull * (uint64_t)c.tile;
        grid = (int)((tiles + per - 1u) / per);
    } else if (c.grid > 0) {
        grid = c.grid;
    } else {
        LaunchCfg c2 = c;
        c2.blocks_needed = (((uint64_t)a.n_seg + (64 / G) - 1u) / (64 / G) + 3u) / 4u;
        grid = pick_grid(seg_tile_kernel<G, P, K, NT>, c2);
    }
    hipLaunchKernelGGL((seg_tile_kernel<G, P, K, NT>), dim3(grid), dim3(256), 0, s, a);
    return hipGetLastError();
}

// The v4 instantiations: (G lanes per segment, P KiB image pieces, K chunks per lane).
#define NETCSUM_TILE_TABLE(X)                                                                       \
    X(1, 2, 3) X(1, 4, 6) X(4, 1, 1) X(4, 2, 2) X(8, 2, 2) X(8, 4, 4) X(16, 4, 4) X(16, 6, 6)       \
    X(16, 8, 8) X(32, 2, 2) X(32, 4, 3) X(32, 4, 4) X(32, 8, 8) X(64, 2, 2) X(64, 4, 4) X(64, 8, 8)

bool tile_supported(int g, int p, int k) {
#define X(G_, P_, K_) if (g == G_ && p == P_ && k == K_) return true;
    NETCSUM_TILE_TABLE(X)
#undef X
    return false;
}

static hipError_t launch_tile_dispatch(const SegBatchArgs& a, const LaunchCfg& c, hipStream_t s) {
#define X(G_, P_, K_)                                                                                \
    if (c.group_lanes == G_ && c.tile_pieces == P_ && c.chunks_per_pass == K_) {                     \
        return c.nt ? launch_tile<G_, P_, K_, true>(a, c, s) : launch_tile<G_, P_, K_, false>(a, c, s); \
    }
    NETCSUM_TILE_TABLE(X)
#undef X
    return hipErrorInvalidValue;
}

thread_local char g_last_launch[256];

const char* last_launch() {
    return g_last_launch;
}

void set_last_launch(const char* desc) {
    snprintf(g_last_launch, sizeof(g_last_launch), "%s", desc);
}

static void note_launch(const LaunchCfg& c, const SegBatchArgs& a) {
    static const char* names[] = {"?", "seg_batch_kernel", "seg_pipe_kernel", "seg_lds_kernel", "seg_tile_kernel",
                                  "seg_small_kernel", "seg_stream_kernel", "seg_hdr_kernel", "seg_hdrstream_kernel"};
    const int kid = (c.kernel >= 1 && c.kernel <= 8) ? c.kernel : 0;
    if (kid == 8) {
        snprintf(g_last_launch, sizeof(g_last_launch), "seg_hdrstream_kernel<M=%u,D=%d%s%s> block=256 hdrs_per_wave=%u",
                 a.seg_len / 4u, c.chunks_per_pass, c.nt ? ",nt" : "", hdr_burst() ? ",burst" : "", c.stream_spw);
        return;
    }
    if (kid == 7) {
        const int h = hdr_lanes_h(a, c.tile);
        const int st = c.chunks_per_pass;                         // as launch_hdr_batch resolves it
        const int S = std::min(st == 3 ? 3 : (st == 4 ? 4 : 2), h == 4 ? 3 : 4);
        const uint32_t tiles = (a.n_seg + 64u * h - 1u) / (64u * h);
        const uint32_t g = c.grid > 0 ? (uint32_t)c.grid : (tiles + 15u) / 16u;
        snprintf(g_last_launch, sizeof(g_last_launch), "seg_hdr_kernel<P=%u,S=%d,H=%d> block=256 grid=%u",
                 hdr_pieces(a, h), S, h, std::max<uint32_t>(1u, std::min<uint32_t>(g, (tiles + 3u) / 4u)));
        return;
    }
    if (kid == 6) {
        if (a.seg_off && c.run_bytes) {
            snprintf(g_last_launch, sizeof(g_last_launch),
                     "seg_stream_varlen_kernel<D=%d%s%s> block=256 segs_per_wave=adaptive(>=%u, ~%u B)",
                     c.chunks_per_pass, (a.pseudo && a.pseudo_len) ? ",pseudo" : "", c.nt ? ",nt" : "",
                     c.stream_spw, c.run_bytes);
            return;
        }
        snprintf(g_last_launch, sizeof(g_last_launch), "%s<D=%d%s%s> block=256 segs_per_wave=%u",
                 a.seg_off ? "seg_stream_varlen_kernel" : "seg_stream_kernel", c.chunks_per_pass,
                 (a.pseudo && a.pseudo_len) ? ",pseudo" : "", c.nt ? ",nt" : "", c.stream_spw);
        return;
    }
    snprintf(g_last_launch, sizeof(g_last_launch), "%s<G=%d,K=%d%s%s%s> block=%d tile=%d grid=%d P=%d",
             names[kid], c.group_lanes, c.chunks_per_pass, a.seg_off ? ",varlen" : ",strided",
             c.nt ? ",nt" : "", "", c.block, c.tile, c.grid, c.tile_pieces);
}

hipError_t launch_seg_batch(const SegBatchArgs& args, const LaunchCfg& c, hipStream_t s) {
    note_launch(c, args);
    SegBatchArgs a = args;
    a.tile = c.tile > 0 ? (uint32_t)c.tile : 0u;
    if (c.kernel == 5) {
        return launch_small_batch(a, c.grid, s);              // K = dwords per segment
    }
    if (c.kernel == 6) {
        return launch_stream_batch(a, c.chunks_per_pass, c.stream_spw, c.nt, s);   // K = pieces in flight
    }
    if (c.kernel == 7) {
        return launch_hdr_batch(a, c.chunks_per_pass, c.tile, c.grid, s);                 // K = tiles in flight
    }
    if (c.kernel == 8) {
        return launch_hdrstream(a, c.chunks_per_pass, c.stream_spw, c.nt, s);            // K = pieces in flight
    }
    if (c.kernel == 4) {
        return launch_tile_dispatch(a, c, s);
    }
    if (c.kernel == 3) {
        if (a.seg_off) {
            return c.nt ? launch_lds_g<true, true>(a, c.group_lanes, c.chunks_per_pass, c, s)
                        : launch_lds_g<true, false>(a, c.group_lanes, c.chunks_per_pass, c, s);
        }
        return c.nt ? launch_lds_g<false, true>(a, c.group_lanes, c.chunks_per_pass, c, s)
                    : launch_lds_g<false, false>(a, c.group_lanes, c.chunks_per_pass, c, s);
    }
    if (c.kernel == 2) {
        if (a.seg_off) {
            return c.nt ? launch_pipe_g<true, true>(a, c.group_lanes, c.chunks_per_pass, c, s)
                        : launch_pipe_g<true, false>(a, c.group_lanes, c.chunks_per_pass, c, s);
        }
        return c.nt ? launch_pipe_g<false, true>(a, c.group_lanes, c.chunks_per_pass, c, s)
                    : launch_pipe_g<false, false>(a, c.group_lanes, c.chunks_per_pass, c, s);
    }
    const int k = c.chunks_per_pass > 4 ? 4 : c.chunks_per_pass;
    return a.seg_off ? launch_seg_g<true>(a, c.group_lanes, k, c, c.nt, s)
                     : launch_seg_g<false>(a, c.group_lanes, k, c, c.nt, s);
}

hipError_t launch_stream_exact(const void* d_p, uint32_t n16, unsigned long long* d_sum, int grid,
                               hipStream_t s, uint32_t tag) {
    hipLaunchKernelGGL(stream_exact_kernel, dim3(grid), dim3(256), 0, s,
                       reinterpret_cast<gu32x4*>(reinterpret_cast<uintptr_t>(d_p)), n16, d_sum, grid == 1 ? 1 : 0,
                       grid == 1 ? tag : 0u);
    return hipGetLastError();
}

hipError_t launch_fill(void* d_buf, uint64_t n_bytes, uint64_t first_byte, uint64_t seed, int pattern, int grid,
                       hipStream_t s) {
    hipLaunchKernelGGL(fill_kernel, dim3(grid), dim3(256), 0, s, static_cast<uint8_t*>(d_buf), n_bytes,
                       first_byte, seed, pattern);
    return hipGetLastError();
}

hipError_t launch_read_stream(const void* d_p, uint64_t n16, unsigned long long* d_sink, int grid, bool nt,
                              hipStream_t s, int variant) {
    if (variant == 1) {
        if (nt) {
            hipLaunchKernelGGL(read_stream_lds_kernel<true>, dim3(grid), dim3(256), 0, s,
                               reinterpret_cast<gu32x4*>(reinterpret_cast<uintptr_t>(d_p)), n16, d_sink);
        } else {
            hipLaunchKernelGGL(read_stream_lds_kernel<false>, dim3(grid), dim3(256), 0, s,
                               reinterpret_cast<gu32x4*>(reinterpret_cast<uintptr_t>(d_p)), n16, d_sink);
        }
        return hipGetLastError();
    }
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
