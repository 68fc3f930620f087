// netcsum_stream.h — building blocks of the "run stream" kernels (a WAVE reads a contiguous run of
// segments / packets as 1-KiB pieces, lane l holding bytes [16l, 16l + 16) of each piece):
// netcsum_stream.hip (segment batches, C2 / C4 / C5) and netcsum_pktstream.hip (IPv4 packet batches).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "netcsum_device.h"

namespace netcsum {
namespace sv {

constexpr int kRsrcWord3 = 0x00020000;     // gfx9-family raw buffer V# word 3 (32-bit data format)
constexpr uint32_t kOOB = 0x80000000u;     // voffset past every run's num_records: reads zeros

__device__ __forceinline__ __amdgpu_buffer_rsrc_t run_rsrc(uintptr_t base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(base), (short)0, (int)bytes, kRsrcWord3);
}

template <bool NT>
__device__ __forceinline__ u32x4 buf_load16(__amdgpu_buffer_rsrc_t r, uint32_t voff) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, 0, NT ? 2 : 0);
}

// `opaque` over the whole 128-bit register tuple (one "+v" operand): the value stays in the tuple the
// load wrote, so the refill of the same ring slot needs no copy (a copy would force a vmcnt wait).
__device__ __forceinline__ u32x4 opaque_tuple(u32x4 v) {
    asm volatile("" : "+v"(v));
    return v;
}

// This lane's share of the bytes of a 1-KiB piece that lie below piece offset x (wave-uniform,
// 0..1024): its whole chunk if the chunk ends at or below x, the low (x - 16*lane) bytes if x falls
// inside it, nothing above. A span [xs, xe) of the piece is prefix(xe) - prefix(xs), exactly.
// s4 = sum4(v, 0), the whole chunk. Only the lane holding byte x masks its chunk, and its byte count
// is x & 15: the two 64-bit masks depend on x alone, so with x uniform they are scalar work and each
// boundary costs the wave 4 AND + 4 SAD + 2 compare + 2 select (the per-lane clamp-and-mask form
// it replaces cost ~35 VALU per boundary; profiles/r3h_instmix_rx_gap.txt).
__device__ __forceinline__ uint32_t piece_prefix(u32x4 v, uint32_t s4, uint32_t lane16, uint32_t x) {
    const uint32_t k = x & 15u;
    const uint64_t m0 = k >= 8u ? ~0ull : (1ull << (8u * k)) - 1ull;
    const uint64_t m1 = k <= 8u ? 0ull : (1ull << (8u * (k - 8u))) - 1ull;
    uint32_t pv = __builtin_amdgcn_sad_u16(v.x & (uint32_t)m0, 0u, 0u);
    pv = __builtin_amdgcn_sad_u16(v.y & (uint32_t)(m0 >> 32), 0u, pv);
    pv = __builtin_amdgcn_sad_u16(v.z & (uint32_t)m1, 0u, pv);
    pv = __builtin_amdgcn_sad_u16(v.w & (uint32_t)(m1 >> 32), 0u, pv);
    return (lane16 + 16u <= x) ? s4 : ((lane16 < x) ? pv : 0u);
}

// Sum over the 64 lanes (every lane active): inclusive row scans by DPP row_shr 1/2/4/8 (lanes with
// no source add the 0 `old` operand), then the four row totals from lanes 15/31/47/63 (scalar).
__device__ __forceinline__ uint32_t wave_total(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 15) + (uint32_t)__builtin_amdgcn_readlane((int)v, 31) +
           (uint32_t)__builtin_amdgcn_readlane((int)v, 47) + (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// Inclusive prefix sum over the 64 lanes (every lane active): the row scans of wave_total, then the
// totals of the rows below added from lanes 15 / 31 / 47.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, uint32_t lane) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);
    const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)v, 15);
    const uint32_t r1 = (uint32_t)__builtin_amdgcn_readlane((int)v, 31);
    const uint32_t r2 = (uint32_t)__builtin_amdgcn_readlane((int)v, 47);
    return v + (lane >= 16u ? r0 : 0u) + (lane >= 32u ? r1 : 0u) + (lane >= 48u ? r2 : 0u);
}

// Row touch. Before streaming its run, a wave loads the first dword of every 1-KiB piece of the run
// (lane q: piece q, and q + 64; plain cache policy) and never uses the values. The stream's own
// loads are non-temporal 1-KiB wave-instructions issued D at a time; the touches put a request into
// every part of the run up front, and the stream's later loads of those lines and their neighbours
// find them under way. Measured on C2 (tools/c2_probe.py, profiles/r2cx_*): 0.2339 -> 0.2260 ms at
// full residency, 0.2174 ms with 5 waves per SIMD; touches every 512 / 256 B or with the nt policy
// are slower. Runs longer than 128 pieces are touched in their first 128 KiB.
struct RunTouch {
    uint32_t a, b;
};

__device__ __forceinline__ RunTouch touch_run(__amdgpu_buffer_rsrc_t r, uint32_t npieces, uint32_t lane, bool on) {
    RunTouch t;
    t.a = __builtin_amdgcn_raw_buffer_load_b32(r, (int)(on && lane < npieces ? lane << 10 : kOOB), 0, 0);
    t.b = __builtin_amdgcn_raw_buffer_load_b32(r, (int)(on && lane + 64u < npieces ? (lane + 64u) << 10 : kOOB), 0, 0);
    return t;
}

// The touched values are consumed here: either after a wait that in-order retirement already makes
// cover the touches (loads issued after them and awaited anyway), or after the run's final vmcnt(0).
// Never earlier: consuming them alone would wait for every piece issued before them.
__device__ __forceinline__ void touch_retire(RunTouch t) {
    asm volatile("" ::"v"(t.a), "v"(t.b));
}

// XCD-aware block order (cdna_hip_programming.md §5.5 T1, bijective form). mode 1: blocks the
// dispatcher places on one XCD (equal blockIdx mod 8) take one contiguous 1/8 of the grid's runs, so
// each XCD's L2 and address translation see one slice of the batch instead of all of it. mode C >= 2
// (round 6): each XCD takes chunks of C consecutive blocks in turn — chunk x, x + 8, x + 16, … — so
// that each XCD still reads contiguous runs while the 8 XCDs stay in one moving window of the batch
// instead of 8 streams a slice apart (blocks past the last whole round of 8 chunks keep their order).
__device__ __forceinline__ uint32_t xcd_block(uint32_t orig, uint32_t nwg, uint32_t mode = 1u) {
    const uint32_t xcd = orig & 7u;
    if (mode <= 1u) {
        const uint32_t q = nwg >> 3, r = nwg & 7u;
        return (xcd < r ? xcd * (q + 1u) : r * (q + 1u) + (xcd - r) * q) + (orig >> 3);
    }
    const uint32_t full = nwg - nwg % (8u * mode);
    if (orig >= full) {
        return orig;
    }
    const uint32_t slot = orig >> 3;
    return ((slot / mode) * 8u + xcd) * mode + slot % mode;
}

}  // namespace sv
}  // namespace netcsum
