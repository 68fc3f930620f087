// netcsum_device.h — device-side building blocks shared by the gfx950 checksum kernels
// (netcsum_kernels.hip: segment batches; netcsum_packets.hip: IPv4 packet batches).
// Arithmetic conventions: see the header comment of netcsum_kernels.hip.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

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

// Rx burst action (NetUtil_MI355X_RxBurst, include/netcsum_mi355x.h (2b'')) of a datagram from its
// NETCSUM_PKT_* verdict `f` and the transport protocol whose checksum the verdict covers. The order
// of the tests is the reference's order of checks: the IPv4 header's shape (MALFORMED, delivered: the
// stack rejects it itself), the IPv4 header checksum (net_ipv4.c:5243-5254), fragments (transport
// verified after reassembly, net_ipv4.c:6523), transport shape (delivered), then the transport
// checksum of each protocol.
__host__ __device__ __forceinline__ uint32_t rx_action(uint32_t f, uint32_t proto, bool v6, uint32_t rx_cfg) {
    if (f & 0x10u) return 0u;                                    // MALFORMED: NETCSUM_RX_DELIVER
    if (!v6 && !(f & 0x01u)) return 1u;                          // IPv4 header checksum failed
    if (f & 0x20u) return 8u;                                    // FRAGMENT: DELIVER_L4_UNVERIFIED
    if (f & 0xC0u) return 0u;                                    // EXT_HDR / L4_MALFORMED: the stack
    if (f & 0x08u) return (rx_cfg & 1u) ? 4u : 0u;               // UDP without a checksum (net_udp.c:1971)
    if ((f & 0x06u) != 0x04u) return 0u;                         // not checked, or checked and valid
    switch (proto) {
    case 6u:  return 2u;                                         // TCP
    case 17u: return 3u;                                         // UDP
    case 1u:  return v6 ? 0u : 5u;                               // ICMPv4
    case 2u:  return v6 ? 0u : 6u;                               // IGMP
    case 58u: return v6 ? 7u : 0u;                               // ICMPv6
    default:  return 0u;
    }
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

// Makes a loaded chunk opaque to the optimiser, so its use cannot be sunk into a branch: every
// CFG path then waits for the load, and no load stays "pending" across a loop back-edge (the
// waitcnt pass would drain vmcnt(0) before the register is re-used, serialising the pipeline).
__device__ __forceinline__ u32x4 opaque(u32x4 v) {
    asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w));
    return v;
}

// Iterations of a group walking first, first + step, ... < end, and the wave-uniform trip count
// (the wave's lane 0 has the smallest `first` of its groups, hence the most iterations). A loop
// over the uniform count with per-group validity keeps exits scalar: a divergent `break` in the
// middle of a software-pipelined loop leaves a CFG path that skips the consume of the in-flight
// stage, which again makes the compiler drain vmcnt(0) at the loop head.
__device__ __forceinline__ uint32_t group_iters(uint32_t first, uint32_t step, uint32_t end) {
    return first < end ? (uint32_t)(((uint64_t)end - first + step - 1u) / step) : 0u;
}

template <int G>
__device__ __forceinline__ uint32_t group_sum(uint32_t s) {
#pragma unroll
    for (int m = G / 2; m >= 1; m >>= 1) {
        s += __shfl_xor(s, m, 64);
    }
    return s;
}

// A 16-byte zero chunk inside the code object (one per translation unit): chunk slots past the
// end of a span load from here, so every load is unconditional and always hits mapped memory.
// 64-B aligned: a frame that starts at the sector below its span (Tx sector write-back) maps the
// zero chunk to lead 0.
static __device__ __attribute__((aligned(64))) u32x4 g_zero_chunk[4];

__device__ __forceinline__ uintptr_t zero_addr() {
    return reinterpret_cast<uintptr_t>(&g_zero_chunk[0]);
}

__device__ __forceinline__ uint32_t span_chunks(uintptr_t a, uint32_t len) {
    return len ? (uint32_t)((a + len - (a & ~(uintptr_t)15) + 15) >> 4) : 0u;
}

// Mask chunk c of a span given in span-relative terms: the span covers bytes [lead, rend) of its
// 16-B-aligned chunk sequence (rend = lead + len). 32-bit arithmetic only.
__device__ __forceinline__ u32x4 edge_mask_rel(u32x4 v, uint32_t c, uint32_t lead, uint32_t rend) {
    const uint32_t q = 16u * c;
    const int lo = (c == 0u) ? (int)lead : 0;
    const int hi = (rend - q < 16u) ? (int)(rend - q) : 16;
    if (lo != 0 || hi != 16) {
        v = mask_chunk(v, lo, hi);
    }
    return v;
}

// Sum of bytes [0, m) of this lane's chunk; m per lane, clamped to [0, 16] (VALU only, no scalar mask work).
__device__ __forceinline__ uint32_t low_bytes(u32x4 v, int m) {
    uint32_t acc = 0u;
    const uint32_t d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int k = min(max(m - 4 * i, 0), 4);
        const uint32_t mask = k >= 4 ? 0xFFFFFFFFu : ((1u << (8 * k)) - 1u);
        acc = __builtin_amdgcn_sad_u16(d[i] & mask, 0u, acc);
    }
    return acc;
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N <= 9, "extend wait_vmcnt");
    if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if constexpr (N == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else if constexpr (N == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if constexpr (N == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
    else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if constexpr (N == 7) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
    else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
}

// Sum (in the absolute LE frame) of the byte span [a, a+len) by the G lanes of a group; K chunks
// per lane per pass. Returns the lane's 32-bit partial (exact for
// spans < 64 KiB).
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

typedef __attribute__((address_space(3))) void lds_void;


}  // namespace netcsum
