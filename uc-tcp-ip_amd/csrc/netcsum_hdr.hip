// netcsum_hdr.hip — gfx950 kernel for batches of SMALL strided headers through an LDS image
// (config C3: 16 M x 20 B IPv4 headers; NetUtil_16BitOnesCplChkSumHdrCalc / ...HdrVerify,
// net_util.c:159-195 / :245-284, whose sum is NetUtil_16BitSumHdrCalc, net_util.c:1160-1208).
//
// H headers per lane (lane l takes headers l, 64 + l, ...), as in seg_small_kernel
// (netcsum_small.hip), but the bytes do not reach the lanes through per-lane 20-B-strided loads: a
// wave's TILE of 64*H consecutive headers is one contiguous byte range, fetched as whole 1-KiB
// LDS-DMA pieces (raw buffer loads with the `lds` modifier: 64 lanes x 16 B, 8 aligned cache lines per
// wave-instruction, the hardware range check drops the lanes past the tile), and each lane then
// reads its headers' ND dwords back from the LDS image (ds_read_b32 at a 4-B-aligned offset; an odd
// dword stride such as 5 is bank-conflict free). H > 1 fills the pieces better: a 64-header tile of
// 20-B headers is 1.26 KiB in two pieces (63 % of the lanes carry bytes), 128 headers 2.5 KiB in
// three (84 %).
//
// Pipeline: each wave keeps S tiles in flight in an LDS ring (S x P KiB per wave). Nothing orders a
// ds_read behind an LDS-DMA except the wave's own vmcnt, so the waits are counted by hand, and they
// count only what is certain to retire after the tile being consumed: the DMAs of the m REAL tiles
// issued after it (loads retire in order among themselves), wait vmcnt(m*P). Stores are not counted
// (they may retire out of order with the loads; counting them could let the wait pass early, not
// counting them can only wait longer), and no dummy loads are issued past a wave's last tile (a load
// whose lanes are all out of range may retire at once). An earlier form that counted H stores and
// dummy tiles per iteration read a not-yet-landed tile about once in 140 runs of a 1025-header batch
// (tools/hdr_race_probe.py).
//
// Tiles are dealt round-robin over the grid's waves (wave g: tiles g, g+W, g+2W, ...), so at any
// time the waves in flight read one dense, advancing window of HBM (the read-probe pattern).
//
// Arithmetic: headers start at even addresses (base and stride multiples of 4), so the
// little-endian half-word sum v_sad_u16 needs no rotation; the last dword is masked to the header's
// length; ~fold16 is the reference's host-order return value (netcsum_kernels.hip header).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "netcsum_device.h"
#include "netcsum_kernels.h"

namespace netcsum {

namespace {

constexpr int kRsrcWord3 = 0x00020000;     // gfx9-family raw buffer V# word 3
constexpr uint32_t kOOB = 0x80000000u;     // offset past every num_records: dropped by the range check

typedef __attribute__((address_space(3))) void lds_t;

// Built from readfirstlane'd inputs so the compiler can prove the V# wave-uniform (else it wraps
// every buffer op in a waterfall loop — cdna_hip_programming.md T20).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t bytes) {
    const uint64_t b = reinterpret_cast<uintptr_t>(base);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    void* p = reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), kRsrcWord3);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
    static_assert(N >= 0 && N <= 63, "vmcnt is 6 bits on gfx9");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// P KiB pieces per tile, S tiles in flight per wave, H headers per lane (64*H per tile).
template <int P, int S, int H>
__global__ void __launch_bounds__(256) seg_hdr_kernel(SegBatchArgs A, uint32_t nd) {
    __shared__ uint32_t img[4][S][P * 256];                    // per wave: S stages x P KiB
    constexpr uint32_t TH = 64u * (uint32_t)H;                 // headers per tile
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t n = A.n_seg;
    const uint32_t ntiles = (n + TH - 1u) / TH;
    const uint32_t W = gridDim.x * 4u;
    const uint32_t t0 = blockIdx.x * 4u + w;
    if (t0 >= ntiles) {
        return;
    }
    const uint32_t cnt = (ntiles - t0 + W - 1u) / W;          // tiles of this wave
    const uint32_t st = (uint32_t)A.seg_stride;
    const uint32_t len = A.seg_len;
    const uint32_t last_mask = (len & 3u) ? ((1u << (8u * (len & 3u))) - 1u) : 0xFFFFFFFFu;
    const uintptr_t base = (uintptr_t)A.base;
    const bool verify = A.verify != 0u;
    const __amdgpu_buffer_rsrc_t ro = rsrc(A.out, verify ? n : 2u * n);

    // Issue tile i (< cnt) into ring slot i % S: always exactly P LDS-DMA loads, every one with at
    // least one in-range lane. A piece wholly past a short (last) tile re-reads piece 0's bytes into
    // its own LDS slot (never read back) instead of issuing an all-out-of-range load, whose return
    // order relative to the other loads is the one thing the hand-counted waits cannot rely on.
    auto issue = [&](uint32_t i) {
        const uint32_t slot = i % (uint32_t)S;
        const uint32_t h0 = (t0 + i * W) * TH;
        const uint32_t nh = min(TH, n - h0);
        const uintptr_t a0 = base + (uint64_t)h0 * st;
        const uintptr_t i0 = a0 & ~(uintptr_t)15;
        const uint32_t bytes = (uint32_t)(a0 - i0) + (nh - 1u) * st + len;
        const __amdgpu_buffer_rsrc_t r = rsrc(reinterpret_cast<const void*>(i0), (bytes + 15u) & ~15u);
#pragma unroll
        for (int p = 0; p < P; ++p) {
            const uint32_t pb = (1024u * (uint32_t)p < bytes) ? 1024u * (uint32_t)p : 0u;   // wave-uniform
            __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_t*)&img[w][slot][p * 256], 16,
                                                     (int)(pb + 16u * lane), 0, 0, 2);
        }
    };

    // Prologue: the first S-1 tiles (those that exist).
#pragma unroll
    for (int j = 0; j < S - 1; ++j) {
        if ((uint32_t)j < cnt) {
            issue((uint32_t)j);
        }
    }
    // Wait counts. Issue order of a wave with cnt tiles: tiles 0..S-2 in the prologue, then tile i+S-1
    // at the top of iteration i (if it exists), P loads each; loads retire in issue order, stores
    // are not counted. When iteration i waits for tile i, the loads issued after tile i's are those of
    // tiles i+1 .. min(i+S-1, cnt-1): m = min(S-1, cnt-1-i) tiles = m*P loads, so vmcnt(m*P) returns
    // exactly when tile i has landed:
    //
    //   S | cnt-1-i >= S-1 (steady) | cnt-1-i = 2   | cnt-1-i = 1 | cnt-1-i = 0 (last tile)
    //   2 | m = 1: vmcnt(P)         |  (steady)     |  (steady)   | m = 0: vmcnt(0)
    //   3 | m = 2: vmcnt(2P)        |  (steady)     | vmcnt(P)    | vmcnt(0)
    //   4 | m = 3: vmcnt(3P)        | vmcnt(2P)     | vmcnt(P)    | vmcnt(0)
    //
    // (a wave with cnt < S tiles starts in the tail columns). tests/test_gpu_hdr_waits.py runs every
    // instance with waves owning exactly 1 .. S+1 tiles, full and short last tiles, against the oracle.
    for (uint32_t i = 0; i < cnt; ++i) {
        if (i + (uint32_t)S - 1u < cnt) {
            issue(i + (uint32_t)S - 1u);
        }
        const uint32_t m = min((uint32_t)S - 1u, cnt - 1u - i);   // real tiles issued after tile i
        if (m == (uint32_t)S - 1u) {                          // tile i landed in LDS
            wait_vm<(S - 1) * P>();
        } else if (m == 2u) {
            wait_vm<(S > 3 ? 2 : 0) * P>();
        } else if (m == 1u) {
            wait_vm<(S > 2 ? 1 : 0) * P>();
        } else {
            wait_vm<0>();
        }
        const uint32_t slot = i % (uint32_t)S;
        const uint32_t h0 = (t0 + i * W) * TH;
        const uint32_t nh = min(TH, n - h0);
        const uintptr_t a0 = base + (uint64_t)h0 * st;
        const uint32_t* im = &img[w][slot][0];
        uint32_t sres[H];
#pragma unroll
        for (int hh = 0; hh < H; ++hh) {
            const uint32_t j = 64u * (uint32_t)hh + lane;      // header within the tile
            const uint32_t dw0 = ((uint32_t)(a0 & 15u) + j * st) >> 2;   // its first dword in the image
            uint32_t acc = 0u;
            for (uint32_t d = 0; d + 1u < nd; ++d) {
                acc = __builtin_amdgcn_sad_u16(im[dw0 + d], 0u, acc);
            }
            acc = __builtin_amdgcn_sad_u16(im[dw0 + nd - 1u] & last_mask, 0u, acc);
            sres[hh] = fold16(acc);
        }
#pragma unroll
        for (int hh = 0; hh < H; ++hh) {
            const uint32_t j = 64u * (uint32_t)hh + lane;
            const uint32_t h = h0 + j;
            const uint32_t s = sres[hh];
            if (verify) {
                __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(s == 0xFFFFu ? 1u : 0u), ro,
                                                     (int)(j < nh ? h : kOOB), 0, 0);
            } else {
                __builtin_amdgcn_raw_buffer_store_b16((uint16_t)(~s), ro, (int)(j < nh ? 2u * h : kOOB), 0, 0);
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");    // image reads done before the slot refills
    }
}

template <int P, int S, int H>
hipError_t launch_hdr_t(const SegBatchArgs& a, int grid, hipStream_t s) {
    const uint32_t tiles = (a.n_seg + 64u * H - 1u) / (64u * H);
    const uint32_t g = grid > 0 ? (uint32_t)grid : (tiles + 15u) / 16u;      // default: 4 tiles per wave
    hipLaunchKernelGGL((seg_hdr_kernel<P, S, H>), dim3(std::max<uint32_t>(1u, std::min<uint32_t>(g, (tiles + 3u) / 4u))),
                       dim3(256), 0, s, a, (a.seg_len + 3u) >> 2);
    return hipGetLastError();
}

}  // namespace

// Pieces per tile of 64*H headers: the image starts at the 16-B boundary below the tile. Base and
// stride are multiples of 4 (small_supported), so a tile spans 64*H*stride = a multiple of 256 bytes
// and EVERY tile starts at the base's offset in its 16-B line (lead = base & 15, 0..12): the exact
// piece count for that lead (C3's 256-header tiles of 20 B are 5 whole KiB at lead 0, not 6).
uint32_t hdr_pieces(const SegBatchArgs& a, int h) {
    const uint64_t lead = (uintptr_t)a.base & 15u;
    return (uint32_t)((lead + (64u * (uint64_t)h - 1u) * a.seg_stride + a.seg_len + 1023u) / 1024u);
}

bool hdr_supported(const SegBatchArgs& a) {
    return small_supported(a) && a.seg_stride <= 64u && hdr_pieces(a, 1) <= 5u && a.n_seg < 0x3FFFFFFFu;
}

// Headers per lane: the requested 1, 2 or 4 where its tile fits 6 pieces; auto (h <= 0) = 2.
int hdr_lanes_h(const SegBatchArgs& a, int h) {
    if (h != 1 && h != 2 && h != 4) h = 2;
    while (h > 1 && hdr_pieces(a, h) > 6u) h >>= 1;
    return h;
}

#define NETCSUM_HDR_LIST(X) \
    X(1, 2, 1) X(1, 3, 1) X(1, 4, 1) X(2, 2, 1) X(2, 3, 1) X(2, 4, 1) X(3, 2, 1) X(3, 3, 1) X(3, 4, 1) \
    X(4, 2, 1) X(4, 3, 1) X(4, 4, 1) X(5, 2, 1) X(5, 3, 1) X(5, 4, 1)                                  \
    X(1, 2, 2) X(1, 3, 2) X(1, 4, 2) X(2, 2, 2) X(2, 3, 2) X(2, 4, 2) X(3, 2, 2) X(3, 3, 2) X(3, 4, 2) \
    X(4, 2, 2) X(4, 3, 2) X(4, 4, 2) X(5, 2, 2) X(5, 3, 2) X(5, 4, 2) X(6, 2, 2) X(6, 3, 2) X(6, 4, 2) \
    X(1, 2, 4) X(1, 3, 4) X(2, 2, 4) X(2, 3, 4) X(3, 2, 4) X(3, 3, 4) X(4, 2, 4) X(4, 3, 4)            \
    X(5, 2, 4) X(5, 3, 4) X(6, 2, 4) X(6, 3, 4)

// Resident 256-thread blocks per CU. stages 2..4 (H = 4: 2..3).
int hdr_occupancy(const SegBatchArgs& a, int stages, int h) {
    h = hdr_lanes_h(a, h);
    const uint32_t p = hdr_pieces(a, h);
    const int S = std::min(stages == 3 ? 3 : (stages == 4 ? 4 : 2), h == 4 ? 3 : 4);
    int occ = 0;
    hipError_t e = hipErrorInvalidValue;
#define NETCSUM_H(P_, S_, H_) \
    if (p == P_ && S == S_ && h == H_) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, seg_hdr_kernel<P_, S_, H_>, 256, 0);
    NETCSUM_HDR_LIST(NETCSUM_H)
#undef NETCSUM_H
    return (e == hipSuccess && occ > 0) ? occ : 1;
}

hipError_t launch_hdr_batch(const SegBatchArgs& a, int stages, int h, int grid, hipStream_t s) {
    if (!hdr_supported(a)) return hipErrorInvalidValue;
    h = hdr_lanes_h(a, h);
    const uint32_t p = hdr_pieces(a, h);
    const int S = std::min(stages == 3 ? 3 : (stages == 4 ? 4 : 2), h == 4 ? 3 : 4);
#define NETCSUM_H(P_, S_, H_) \
    if (p == P_ && S == S_ && h == H_) return launch_hdr_t<P_, S_, H_>(a, grid, s);
    NETCSUM_HDR_LIST(NETCSUM_H)
#undef NETCSUM_H
    return hipErrorInvalidValue;
}

}  // namespace netcsum
