// netcsum_crc.hip — gfx950 CRC-32 of µC/TCP-IP's Source/net_util.c:485-636: the IEEE 802.3
// polynomial in reflected form (0xEDB88320, net_util.c:77), register initialised to 0xFFFFFFFF
// (NET_UTIL_32_BIT_ONES_CPL_NEG_ZERO, :58), octets shifted in LSB first (:510-524);
// NetUtil_32BitCRC_Calc returns the register as is, NetUtil_32BitCRC_CalcCpl complemented (:583).
// The reference's callers hash 6-byte multicast MAC addresses (Dev/Ether/*/net_dev_*.c,
// AddrMulticastAdd / Remove); the batch form here takes any number of segments of any length.
//
// Arithmetic. The register update is linear over GF(2). Write A^n for "advance the register over n
// zero octets" (a linear map: multiplication by x^(8n) modulo the polynomial). Processing octets M
// from state I gives A^|M|(I) xor raw(M), raw() = the CRC from state 0, and raw() of leading zero
// octets is 0. Any linear map of the 32-bit register is four 256-entry tables, one per register
// octet: A^n(c) = S[0][c & 0xFF] ^ S[1][(c >> 8) & 0xFF] ^ S[2][(c >> 16) & 0xFF] ^ S[3][c >> 24]
// with S[k][b] = A^n(b << 8k). The four octets of a little-endian dword w enter the register
// together: c <- A^4(c ^ w) (slicing-by-4; T = the tables of A^4, T[3] = the byte table of the
// reference's bit loop).
//
// Interleaved chunks (crc_ilv_kernel<G>, segments of 32 B and more). A G-lane group (G = 4, 8, 16
// by segment length) owns a segment. The segment's bytes from the 16-B line at or below its start
// up to the last 16-B boundary at or below its end are 16-B chunks, front-padded with zero chunks to
// G M chunks; lane l takes chunks l, l + G, l + 2G, ... The lane's register runs over its chunk's
// first three dwords with T and over the fourth with Z = A^(16 (G - 1)) o A^4, i.e. it is carried
// past the G - 1 chunks the other lanes own, so that it stands at the start of the lane's next
// chunk; the last chunk uses T, which leaves lane l at the end of chunk l + G (M - 1). log2(G)
// shuffle levels then merge pairs of lanes 16, 32, 64, 128 B apart (tables of A^16 .. A^128), giving
// raw() of the chunk area in lane G - 1, which finishes the < 16 trailing octets alone. Every global load is a whole aligned 16-B chunk, a group's load
// instruction reads 256 contiguous bytes, and every step of every lane is four independent table
// lookups in LDS: no GF(2) multiplications at run time. The bytes of the first line below the
// segment start are masked to zero, and the reference's initial register 0xFFFFFFFF enters as an
// xor into the segment's first four octets (for a message of at least 4 octets, the initial register
// and an xor of its first four octets are the same thing).
//
// Block combine (crc_group_kernel, the round-2 form, kept as NETCSUM_TUNE_CRC_KERNEL 1): lane j of
// a 16-lane group runs over block j of the segment's equal blocks (byte-aligned, v_alignbyte_b32
// windows) and the group merges the blocks by GF(2) multiplications with x^(8 s 2^k) computed by a
// 32-step bit loop. Short segments (<= kCrcShortMax, strided) take one lane each (crc_lane_kernel).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <atomic>
#include <string>
#include <vector>

#include "netcsum_device.h"
#include "netcsum_kernels.h"

namespace netcsum {

namespace {

constexpr uint32_t kPoly = 0xEDB88320u;

// ---- compile-time tables -----------------------------------------------------------------------
// Table sets of the linear maps used by the kernels, S[k][b] = A^n(b << 8k):
enum : int {
    kSetT = 0,                          // A^4 (slicing-by-4; [3] = the byte table)
    kSet16 = 1, kSet32 = 2, kSet64 = 3, kSet128 = 4,   // A^16 .. A^128: the combine levels
    kSetZ16 = 5, kSetZ8 = 6, kSetZ4 = 7, kSetZ2 = 8,   // A^(16 (G - 1)) o A^4 for G = 16, 8, 4, 2 lanes
    kNumSets = 9
};

struct CrcTabs {
    uint32_t s[kNumSets][4][256];
};

struct Set {
    uint32_t t[4][256];
};

constexpr uint32_t zero_octet(uint32_t c) {                     // A^1 by the reference's bit loop
    for (int j = 0; j < 8; ++j) {
        c = (c & 1u) ? ((c >> 1) ^ kPoly) : (c >> 1);
    }
    return c;
}

constexpr uint32_t apply_set(const Set& S, uint32_t c) {
    return S.t[0][c & 0xFFu] ^ S.t[1][(c >> 8) & 0xFFu] ^ S.t[2][(c >> 16) & 0xFFu] ^ S.t[3][c >> 24];
}

constexpr Set compose(const Set& outer, const Set& inner) {    // tables of outer o inner
    Set r{};
    for (int k = 0; k < 4; ++k) {
        for (int b = 0; b < 256; ++b) {
            r.t[k][b] = apply_set(outer, inner.t[k][b]);
        }
    }
    return r;
}

constexpr CrcTabs make_tabs() {
    Set t4{};
    for (int k = 0; k < 4; ++k) {
        for (uint32_t b = 0; b < 256u; ++b) {
            uint32_t c = b << (8 * k);
            for (int j = 0; j < 4; ++j) {
                c = zero_octet(c);
            }
            t4.t[k][b] = c;
        }
    }
    const Set t8 = compose(t4, t4);
    const Set t16 = compose(t8, t8);
    const Set t32 = compose(t16, t16);
    const Set t64 = compose(t32, t32);
    const Set t128 = compose(t64, t64);
    const Set z16 = compose(t128, compose(t64, compose(t32, compose(t16, t4))));   // A^(240 + 4)
    const Set z8 = compose(t64, compose(t32, compose(t16, t4)));                   // A^(112 + 4)
    const Set z4 = compose(t32, compose(t16, t4));                                 // A^(48 + 4)
    const Set z2 = compose(t16, t4);                                               // A^(16 + 4)
    const Set* sets[kNumSets] = {&t4, &t16, &t32, &t64, &t128, &z16, &z8, &z4, &z2};
    CrcTabs r{};
    for (int s = 0; s < kNumSets; ++s) {
        for (int k = 0; k < 4; ++k) {
            for (int b = 0; b < 256; ++b) {
                r.s[s][k][b] = sets[s]->t[k][b];
            }
        }
    }
    return r;
}

__device__ const CrcTabs kTabs = make_tabs();

// 11-bit slicing: the same linear maps as three tables indexed by register bits [0, 11), [11, 22)
// and [22, 32): 3 LDS lookups per dword instead of 4 (20 KiB per map).
constexpr int kWide = 5120;
enum : int { kWideT = 0, kWideZ16 = 1, kWideZ8 = 2, kWideZ4 = 3, kWideZ2 = 4, kNumWide = 5 };

struct CrcWide {
    uint32_t w[kNumWide][kWide];
};

constexpr CrcWide make_wide() {
    const CrcTabs t = make_tabs();
    const int src[kNumWide] = {kSetT, kSetZ16, kSetZ8, kSetZ4, kSetZ2};
    CrcWide r{};
    for (int m = 0; m < kNumWide; ++m) {
        const uint32_t(&S)[4][256] = t.s[src[m]];
        auto ap = [&](uint32_t c) {
            return S[0][c & 0xFFu] ^ S[1][(c >> 8) & 0xFFu] ^ S[2][(c >> 16) & 0xFFu] ^ S[3][c >> 24];
        };
        for (uint32_t b = 0; b < 2048u; ++b) {
            r.w[m][b] = ap(b);
            r.w[m][2048 + b] = ap(b << 11);
        }
        for (uint32_t b = 0; b < 1024u; ++b) {
            r.w[m][4096 + b] = ap(b << 22);
        }
    }
    return r;
}

__device__ const CrcWide kWideTabs = make_wide();

// 6-bit slicing with lane-private replicas (conflict-free): six tables indexed by register bits
// [0, 6), [6, 12), .., [24, 30) and [30, 32) (64, .., 64, 4 entries, 324 in all). ds_read_b32 serves a
// wave in two 32-lane groups and its bank is (address / 4) mod 32 (MI355X_MICROARCH.md, LDS table),
// so LDS entry e of a map is stored 32 times, lane l's copy at word 32 e + (l mod 32): the 32 lanes
// of a group always hit 32 different banks, whatever their indices. 40.5 KiB per map in LDS; random
// lookups into the byte / 11-bit tables cost 6.4 LDS cycles per instruction, 4.4 of them bank
// conflicts (profiles/r2zd_crc_lds_pmc.json), these 2.
constexpr int kK6 = 324;
constexpr int kK6Lds = kK6 * 32;                                // words per replicated map

struct CrcK6 {
    uint32_t m[kNumWide][kK6];
};

constexpr CrcK6 make_k6() {
    const CrcTabs t = make_tabs();
    const int src[kNumWide] = {kSetT, kSetZ16, kSetZ8, kSetZ4, kSetZ2};
    CrcK6 r{};
    for (int m = 0; m < kNumWide; ++m) {
        const uint32_t(&S)[4][256] = t.s[src[m]];
        auto ap = [&](uint32_t c) {
            return S[0][c & 0xFFu] ^ S[1][(c >> 8) & 0xFFu] ^ S[2][(c >> 16) & 0xFFu] ^ S[3][c >> 24];
        };
        for (int j = 0; j < 6; ++j) {
            for (uint32_t e = 0; e < (j < 5 ? 64u : 4u); ++e) {
                r.m[m][64 * j + (int)e] = ap(e << (6 * j));
            }
        }
    }
    return r;
}

__device__ const CrcK6 kK6Tabs = make_k6();

// Replicate map m of kK6Tabs into dst (kK6Lds words). No barrier: the caller's.
template <int B>
__device__ __forceinline__ void fill_k6(uint32_t* dst, int m) {
    for (int i = (int)threadIdx.x; i < kK6Lds; i += B) {
        dst[i] = kK6Tabs.m[m][i >> 5];
    }
}

// R = the map's replica base + (lane mod 32): six conflict-free lookups.
__device__ __forceinline__ uint32_t apply_k6(const uint32_t* R, uint32_t c) {
    return R[32u * (c & 63u)] ^ R[32u * (64u + ((c >> 6) & 63u))] ^ R[32u * (128u + ((c >> 12) & 63u))] ^
           R[32u * (192u + ((c >> 18) & 63u))] ^ R[32u * (256u + ((c >> 24) & 63u))] ^ R[32u * (320u + (c >> 30))];
}
static_assert(make_tabs().s[kSetT][3][1] == 0x77073096u, "byte table of the reflected IEEE polynomial");
static_assert(make_tabs().s[kSetT][3][255] == 0x2D02EF8Du, "byte table of the reflected IEEE polynomial");

// Copy table sets into LDS: sets [0, n) to slots [0, n) and, if z >= 0, set z to slot n
// (blockDim.x == B; one uint4 = 16 B per thread and step). No barrier: the caller's.
template <int B = 256>
__device__ __forceinline__ void copy_sets(uint32_t (*L)[4][256], int n, int z) {
    const uint4* src = reinterpret_cast<const uint4*>(&kTabs.s[0][0][0]);
    uint4* dst = reinterpret_cast<uint4*>(&L[0][0][0]);
    for (int i = (int)threadIdx.x; i < n * 256; i += B) {
        dst[i] = src[i];
    }
    if (z >= 0) {
        for (int i = (int)threadIdx.x; i < 256; i += B) {
            dst[n * 256 + i] = src[z * 256 + i];
        }
    }
}

__device__ __forceinline__ void load_sets(uint32_t (*L)[4][256], int n, int z) {
    copy_sets<256>(L, n, z);
    __syncthreads();
}

template <int B>
__device__ __forceinline__ void copy_wide(uint32_t* dst_w, int m) {
    const uint4* src = reinterpret_cast<const uint4*>(&kWideTabs.w[m][0]);
    uint4* dst = reinterpret_cast<uint4*>(dst_w);
    for (int i = (int)threadIdx.x; i < kWide / 4; i += B) {
        dst[i] = src[i];
    }
}

__device__ __forceinline__ uint32_t apply_wide(const uint32_t* W, uint32_t c) {
    return W[c & 0x7FFu] ^ W[2048u + ((c >> 11) & 0x7FFu)] ^ W[4096u + (c >> 22)];
}

__device__ __forceinline__ uint32_t apply(const uint32_t (*S)[256], uint32_t c) {
    return S[0][c & 0xFFu] ^ S[1][(c >> 8) & 0xFFu] ^ S[2][(c >> 16) & 0xFFu] ^ S[3][c >> 24];
}

__device__ __forceinline__ uint32_t crc_word(const uint32_t (*T)[256], uint32_t c, uint32_t w) {   // 4 octets, LE
    return apply(T, c ^ w);
}

__device__ __forceinline__ uint32_t crc_byte(const uint32_t (*T)[256], uint32_t c, uint32_t b) {
    return T[3][(c ^ b) & 0xFFu] ^ (c >> 8);
}

__device__ __forceinline__ uint32_t ovr(uint32_t x) {          // opaque register value (see below)
    asm volatile("" : "+v"(x));
    return x;
}

// Dword i (0..3) of the 16 stream bytes starting `sh` bytes into the 32-byte window [a, b]: a
// select chain over opaque register values (a select between array elements is turned into an
// indexed access, which puts the window in scratch memory).
__device__ __forceinline__ uint32_t win16_dword(const uint4& a, const uint4& b, uint32_t sh, int i) {
    const uint32_t j = (sh >> 2) + (uint32_t)i;                 // 0..6
    const uint32_t w0 = ovr(a.x), w1 = ovr(a.y), w2 = ovr(a.z), w3 = ovr(a.w);
    const uint32_t w4 = ovr(b.x), w5 = ovr(b.y), w6 = ovr(b.z), w7 = ovr(b.w);
    const uint32_t lo = j == 0u ? w0 : j == 1u ? w1 : j == 2u ? w2 : j == 3u ? w3 : j == 4u ? w4 : j == 5u ? w5 : w6;
    const uint32_t hi = j == 0u ? w1 : j == 1u ? w2 : j == 2u ? w3 : j == 3u ? w4 : j == 4u ? w5 : j == 5u ? w6 : w7;
    return __builtin_amdgcn_alignbyte(hi, lo, sh & 3u);
}

__device__ __forceinline__ uint32_t crc_16(const uint32_t (*T)[256], uint32_t c, const uint4& a, const uint4& b,
                                           uint32_t sh) {
    c = crc_word(T, c, win16_dword(a, b, sh, 0));
    c = crc_word(T, c, win16_dword(a, b, sh, 1));
    c = crc_word(T, c, win16_dword(a, b, sh, 2));
    return crc_word(T, c, win16_dword(a, b, sh, 3));
}

// Register c advanced over the rem <= 16 octets starting sh bytes into the 32-B window [v0, v1].
__device__ __forceinline__ uint32_t crc_window(const uint32_t (*T)[256], uint32_t c, const uint4& v0, const uint4& v1,
                                               uint32_t sh, uint32_t rem) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t lo = 4u * (uint32_t)i;
        if (lo < rem) {
            const uint32_t w = win16_dword(v0, v1, sh, i);
            if (lo + 4u <= rem) {
                c = crc_word(T, c, w);
            } else {
#pragma unroll
                for (int b = 0; b < 3; ++b) {
                    if (lo + (uint32_t)b < rem) {
                        c = crc_byte(T, c, (w >> (8 * b)) & 0xFFu);
                    }
                }
            }
        }
    }
    return c;
}

// Register c advanced over bytes [p, p + n): whole ALIGNED 16-B loads (a chunk holding any byte of
// the range lies in the range's pages, so reading all of it cannot fault), 64 B of the range per
// step from five loads issued together, the stream's dwords cut out by v_alignbyte_b32; the last
// n mod 16 octets from their chunk(s) in registers. (A per-byte head loop with a load per octet
// made the lanes wait on one dependent load after another: 1.75 ms for 1 M x 1500 B.)
__device__ uint32_t crc_range(const uint32_t (*T)[256], uint32_t c, const uint8_t* p, uint32_t n) {
    const uintptr_t a = (uintptr_t)p;
    const uint32_t sh = (uint32_t)(a & 15u);
    const uint4* q = reinterpret_cast<const uint4*>(a - sh);
    uint32_t done = 0u;
    for (; done + 64u <= n; done += 64u, q += 4) {
        const uint4 v0 = q[0], v1 = q[1], v2 = q[2], v3 = q[3];
        const uint4 v4 = q[sh != 0u ? 4 : 3];                  // not read past the range when aligned
        c = crc_16(T, c, v0, v1, sh);
        c = crc_16(T, c, v1, v2, sh);
        c = crc_16(T, c, v2, v3, sh);
        c = crc_16(T, c, v3, v4, sh);
    }
    for (; done + 16u <= n; done += 16u, ++q) {
        const uint4 v0 = q[0];
        const uint4 v1 = q[sh != 0u ? 1 : 0];
        c = crc_16(T, c, v0, v1, sh);
    }
    // the last n mod 16 octets: from the one or two aligned chunks that hold them (a load per octet
    // made 16 M 6-B MAC addresses TA-bound: six byte loads per lane)
    const uint32_t rem = n - done;
    if (rem != 0u) {
        const uint4 v0 = q[0];
        const uint4 v1 = q[sh + rem > 16u ? 1 : 0];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t lo = 4u * (uint32_t)i;
            if (lo < rem) {
                const uint32_t w = win16_dword(v0, v1, sh, i);
                if (lo + 4u <= rem) {
                    c = crc_word(T, c, w);
                } else {
#pragma unroll
                    for (int b = 0; b < 3; ++b) {
                        if (lo + (uint32_t)b < rem) {
                            c = crc_byte(T, c, (w >> (8 * b)) & 0xFFu);
                        }
                    }
                }
            }
        }
    }
    return c;
}

__device__ __forceinline__ void seg_desc(const CrcBatchArgs& A, uint32_t i, const uint8_t*& p, uint32_t& len) {
    p = A.base + (A.off ? A.off[i] : (uint64_t)i * A.stride);
    len = A.lens ? A.lens[i] : A.len;
}

__device__ __forceinline__ uint32_t crc_finish(uint32_t c, uint32_t len, bool cpl) {
    // an empty segment is the reference's NET_UTIL_ERR_NULL_SIZE case: 0
    return len == 0u ? 0u : (cpl ? ~c : c);
}

// One lane per segment (short segments, e.g. 6-B MAC addresses). Persistent blocks: the tables are
// copied once per block, which then walks its share of the batch 256 segments at a time.
__global__ void __launch_bounds__(256) crc_lane_kernel(CrcBatchArgs A) {
    __shared__ uint32_t L[1][4][256];
    load_sets(L, 1, -1);
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < A.n; i += gridDim.x * 256u) {
        const uint8_t* p;
        uint32_t len;
        seg_desc(A, i, p, len);
        A.out[i] = crc_finish(crc_range(L[0], 0xFFFFFFFFu, p, len), len, A.cpl != 0u);
    }
}

// Strided segments of <= 16 B (the drivers' 6-B MAC addresses): one lane each, and the two aligned
// chunks of the lane's NEXT segment are loaded before its current one is computed (one load round
// trip per segment otherwise bounds the persistent loop: 0.0645 ms for 16 M MACs, 0.0416 with it).
// The address of a segment past the batch is clamped to the current one, so every load is issued on
// every path; global (not flat) loads, since a flat load is waited for with lgkmcnt(0) at once.
__global__ void __launch_bounds__(256) crc_tiny_kernel(CrcBatchArgs A) {
    __shared__ uint32_t L[1][4][256];
    load_sets(L, 1, -1);
    const uint32_t step = gridDim.x * 256u;
    const uint32_t i0 = blockIdx.x * 256u + threadIdx.x;
    auto win = [&](uint32_t i, u32x4& v0, u32x4& v1) {
        const uintptr_t a = (uintptr_t)(A.base + (uint64_t)i * A.stride);
        const uintptr_t q = a & ~(uintptr_t)15u;
        v0 = load16<false>(reinterpret_cast<gu32x4*>(q));
        v1 = load16<false>(reinterpret_cast<gu32x4*>(q + ((a & 15u) + A.len > 16u ? 16u : 0u)));
    };
    auto emit = [&](uint32_t i, const u32x4& v0, const u32x4& v1) {
        const uint32_t sh = (uint32_t)((uintptr_t)(A.base + (uint64_t)i * A.stride) & 15u);
        const uint4 w0{v0.x, v0.y, v0.z, v0.w}, w1{v1.x, v1.y, v1.z, v1.w};
        A.out[i] = crc_finish(crc_window(L[0], 0xFFFFFFFFu, w0, w1, sh, A.len), A.len, A.cpl != 0u);
    };
    if (i0 >= A.n) {
        return;
    }
    if (A.len == 0u) {                 // empty segments (the base may be NULL then): 0, nothing read
        for (uint32_t i = i0; i < A.n; i += step) {
            A.out[i] = 0u;
        }
        return;
    }
    // two segments per trip in alternating registers (a copy of a register a load is still filling
    // would wait for that load)
    u32x4 a0, a1, b0, b1;
    win(i0, a0, a1);
    for (uint32_t i = i0; i < A.n; i += 2u * step) {
        const uint32_t j = i + step, k = i + 2u * step;
        win(j < A.n ? j : i, b0, b1);
        emit(i, a0, a1);
        win(k < A.n ? k : i, a0, a1);
        if (j < A.n) {
            emit(j, b0, b1);
        }
    }
}

constexpr int kG = 16;                  // lanes per segment of the block-combine kernel

// ---- interleaved chunks ------------------------------------------------------------------------
// The masks that make the segment's head chunk q (0 or 1; its other chunks are not touched) enter
// the CRC as the reference sees it: the bytes below the segment start zeroed (q == 0), the initial
// register xored into the segment's first 4 octets (chunk-relative offsets [lead - 16 q, + 4)).
struct HeadMask {
    uint32_t keep[4];
    uint32_t flip[4];
};

__device__ __forceinline__ HeadMask head_mask(int q, int lead) {
    HeadMask h;
    const int s = lead - 16 * q;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        h.keep[j] = q == 0 ? dword_mask(lead, 16, 4 * j) : 0xFFFFFFFFu;
        h.flip[j] = (q == 0 || q == 1) ? dword_mask(s, s + 4, 4 * j) : 0u;
    }
    return h;
}

__device__ __forceinline__ u32x4 apply_head(u32x4 v, const HeadMask& h) {
    v.x = (v.x & h.keep[0]) ^ h.flip[0];
    v.y = (v.y & h.keep[1]) ^ h.flip[1];
    v.z = (v.z & h.keep[2]) ^ h.flip[2];
    v.w = (v.w & h.keep[3]) ^ h.flip[3];
    return v;
}

// The register advanced over the r < 16 octets of the aligned chunk v (the segment's tail).
__device__ __forceinline__ uint32_t crc_tail(const uint32_t (*T)[256], uint32_t c, u32x4 v, uint32_t r) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t lo = 4u * (uint32_t)j;
        if (lo + 4u <= r) {
            c = crc_word(T, c, w[j]);
        } else if (lo < r) {
#pragma unroll
            for (int b = 0; b < 3; ++b) {
                if (lo + (uint32_t)b < r) {
                    c = crc_byte(T, c, (w[j] >> (8 * b)) & 0xFFu);
                }
            }
        }
    }
    return c;
}

constexpr int kRound = 4;               // chunks per lane per round (one round prefetched)

constexpr int log2i(int g) { return g <= 1 ? 0 : 1 + log2i(g / 2); }

// Table form of the chunk steps: W = 0 byte tables (256-thread blocks), 1 11-bit tables (512),
// 2 lane-replicated 6-bit tables (1024; one block per CU).
constexpr uint32_t ilv_block(int w) { return w == 2 ? 1024u : w == 1 ? 512u : 256u; }

template <int G, bool NT, int W>
__global__ void __launch_bounds__(ilv_block(W)) crc_ilv_kernel(CrcBatchArgs A) {
    constexpr uint32_t B = ilv_block(W);
    constexpr int kLevels = log2i(G);                           // combine levels: A^16 .. A^(8 G)
    constexpr int kZ = kLevels + 1;                             // LDS slot of this G's Z (byte tables)
    constexpr int kZset = G == 16 ? kSetZ16 : G == 8 ? kSetZ8 : G == 4 ? kSetZ4 : G == 2 ? kSetZ2 : kSetT;
    constexpr int kZwide = G == 16 ? kWideZ16 : G == 8 ? kWideZ8 : G == 4 ? kWideZ4 : G == 2 ? kWideZ2 : kWideT;
    // byte tables: T, A^16.., Z (8 .. 24 KiB); W 1: T, A^16.. + 2 x 20 KiB; W 2: T, A^16.. + 2 x 40.5 KiB
    constexpr int kWords = W == 2 ? kK6Lds : W == 1 ? kWide : 1;
    __shared__ uint32_t L[W != 0 ? kLevels + 1 : kLevels + 2][4][256];
    __shared__ uint32_t LW[W != 0 ? 2 : 1][kWords];
    copy_sets<B>(L, kLevels + 1, W != 0 ? -1 : kZset);
    if constexpr (W == 1) {
        copy_wide<B>(LW[0], kWideT);
        copy_wide<B>(LW[1], kZwide);
    } else if constexpr (W == 2) {
        fill_k6<B>(LW[0], kWideT);
        fill_k6<B>(LW[1], kZwide);
    }
    __syncthreads();
    const uint32_t* RT = &LW[0][threadIdx.x & 31u];             // W 2: this lane's replicas
    const uint32_t* RZ = &LW[W != 0 ? 1 : 0][threadIdx.x & 31u];
    auto step = [&](uint32_t c, uint32_t w, bool last) -> uint32_t {   // T (last) or Z on c ^ w
        if constexpr (W == 2) {
            return apply_k6(last ? RT : RZ, c ^ w);
        } else if constexpr (W == 1) {
            return apply_wide(last ? LW[0] : LW[1], c ^ w);
        } else {
            return crc_word(last ? L[0] : L[kZ], c, w);
        }
    };
    auto step_t = [&](uint32_t c, uint32_t w) -> uint32_t {
        if constexpr (W == 2) {
            return apply_k6(RT, c ^ w);
        } else if constexpr (W == 1) {
            return apply_wide(LW[0], c ^ w);
        } else {
            return crc_word(L[0], c, w);
        }
    };
    const uint32_t lane = threadIdx.x & (G - 1);
    const uint32_t steps = (A.n + (B / G) - 1u) / (B / G);
    // rounds per segment: wave-uniform for strided batches (bound from the common length)
    const int r_strided = (int)(((A.len + 15u) / 16u + G * kRound - 1u) / (G * kRound));
    for (uint32_t st = blockIdx.x; st < steps; st += gridDim.x) {          // block-uniform trip count
        const uint32_t i = st * (B / G) + threadIdx.x / G;
        const uint8_t* p = A.base;
        uint32_t len = 0u;
        if (i < A.n) {
            seg_desc(A, i, p, len);
        }
        uint32_t c;
        if (len >= 32u) {                                                   // group-uniform
            const uintptr_t a = (uintptr_t)p;
            const uintptr_t fs = a & ~(uintptr_t)15u;
            const uintptr_t e = a + len;
            const uintptr_t ce = e & ~(uintptr_t)15u;
            const uint32_t r = (uint32_t)(e - ce);                          // tail octets, < 16
            const int kc = (int)((ce - fs) >> 4);                           // whole chunks, >= 2
            const int m_n = (kc + G - 1) / G;                               // chunks per lane
            const int pad = m_n * G - kc;                                   // zero chunks in front, < G
            const int lead = (int)(a - fs);
            const int rounds = A.lens ? (m_n + kRound - 1) / kRound : r_strided;
            // Chunk m of this lane is q = lane + G m - pad. A missing one (q < 0: the zero chunks in
            // front, whose register stays 0; m >= m_n: past the lane's last chunk) is loaded from the
            // first chunk (always present) and its steps are discarded by a select on the register,
            // never on the loaded value (a select on it would pull the prefetch's wait forward).
            const int q0 = (int)lane - pad;
            auto fetch = [&](int m) -> u32x4 {
                const int q = q0 + G * m;
                const bool ok = q >= 0 && m < m_n;
                return load16<NT>(reinterpret_cast<gu32x4*>(fs + (ok ? 16u * (uint32_t)q : 0u)));
            };
            u32x4 cur[kRound];
#pragma unroll
            for (int j = 0; j < kRound; ++j) {
                cur[j] = fetch(j);
            }
            const u32x4 tail = load16<NT>(reinterpret_cast<gu32x4*>(r != 0u ? ce : fs));
            // chunks 0 and 1 are the m = 0 chunks of lanes pad and pad + 1, or chunk 1 is the m = 1
            // chunk of lane 0 when pad = G - 1 (G = 1: both are lane 0's, m = 0 and 1)
            const int mh = q0 == 1 - G ? 1 : 0;
            const HeadMask hm = head_mask(q0 + G * mh, lead);
            [[maybe_unused]] HeadMask hm1;
            if constexpr (G == 1) {
                hm1 = head_mask(1, lead);
            }
            c = 0u;
            for (int rd = 0; rd < rounds; ++rd) {
                u32x4 nxt[kRound];
#pragma unroll
                for (int j = 0; j < kRound; ++j) {
                    nxt[j] = fetch(kRound * (rd + 1) + j);
                }
                if (rd == 0) {
                    if constexpr (G == 1) {
                        cur[0] = apply_head(cur[0], head_mask(0, lead));
                        cur[1] = apply_head(cur[1], hm1);
                    } else {
                        cur[0] = mh == 0 ? apply_head(cur[0], hm) : cur[0];
                        cur[1] = mh == 1 ? apply_head(cur[1], hm) : cur[1];
                    }
                }
#pragma unroll
                for (int j = 0; j < kRound; ++j) {
                    const int m = kRound * rd + j;
                    uint32_t t = step_t(c, cur[j].x);
                    t = step_t(t, cur[j].y);
                    t = step_t(t, cur[j].z);
                    t = step(t, cur[j].w, m + 1 == m_n);
                    c = (m < m_n && q0 + G * m >= 0) ? t : c;
                }
#pragma unroll
                for (int j = 0; j < kRound; ++j) {
                    cur[j] = nxt[j];
                }
            }
            // level k: lane j with j % 2d == 2d - 1 (d = 2^k) takes A^(16 d)(c[j - d]) ^ c[j]
#pragma unroll
            for (int k = 0, d = 1; d < G; ++k, d <<= 1) {
                const uint32_t left = (uint32_t)__shfl_up((int)c, d, G);
                if ((lane & (2u * d - 1u)) == 2u * d - 1u) {
                    c ^= apply(L[1 + k], left);
                }
            }
            c = crc_tail(L[0], c, tail, r);
        } else {
            c = lane == G - 1 ? crc_range(L[0], 0xFFFFFFFFu, p, len) : 0u;
        }
        if (i < A.n && lane == G - 1) {
            A.out[i] = crc_finish(c, len, A.cpl != 0u);
        }
    }
}

// ---- block combine (round 2) -------------------------------------------------------------------
// x^(2^k) mod P, reflected (bit 31 = x^0); kX2n[0] = x.
__constant__ uint32_t kX2n[32] = {
    0x40000000u, 0x20000000u, 0x08000000u, 0x00800000u, 0x00008000u, 0xEDB88320u, 0xB1E6B092u, 0xA06A2517u,
    0xED627DAEu, 0x88D14467u, 0xD7BBFE6Au, 0xEC447F11u, 0x8E7EA170u, 0x6427800Eu, 0x4D47BAE0u, 0x09FE548Fu,
    0x83852D0Fu, 0x30362F1Au, 0x7B5A9CC3u, 0x31FEC169u, 0x9FEC022Au, 0x6C8DEDC4u, 0x15D6874Du, 0x5FDE7A4Eu,
    0xBAD90E37u, 0x2E4E5EEFu, 0x4EABA214u, 0xA8A472C0u, 0x429A969Eu, 0x148D302Au, 0xC40BA6D0u, 0xC4E22C3Cu};

// a * b mod P (reflected), fixed trip count (no divergence across the group).
__device__ __forceinline__ uint32_t multmodp(uint32_t a, uint32_t b) {
    uint32_t p = 0u;
#pragma unroll 4
    for (int i = 31; i >= 0; --i) {
        p ^= ((a >> i) & 1u) ? b : 0u;
        b = (b & 1u) ? ((b >> 1) ^ kPoly) : (b >> 1);
    }
    return p;
}

// x^(8 n) mod P.
__device__ __forceinline__ uint32_t x8n(uint32_t n) {
    uint32_t p = 0x80000000u;                                   // x^0
    for (int k = 3; n != 0u; n >>= 1, ++k) {
        if (n & 1u) {
            p = multmodp(kX2n[k & 31], p);
        }
    }
    return p;
}

// A 16-lane group per segment (4 segments per wave, 16 per block and step), persistent blocks.
__global__ void __launch_bounds__(256) crc_group_kernel(CrcBatchArgs A) {
    __shared__ uint32_t L[1][4][256];
    load_sets(L, 1, -1);
    const uint32_t lane = threadIdx.x & (kG - 1);
    const uint32_t steps = (A.n + (256u / kG) - 1u) / (256u / kG);
    for (uint32_t st = blockIdx.x; st < steps; st += gridDim.x) {          // block-uniform trip count
        const uint32_t i = st * (256u / kG) + threadIdx.x / kG;
        const bool valid = i < A.n;
        const uint8_t* p = A.base;
        uint32_t len = 0u;
        if (valid) {
            seg_desc(A, i, p, len);
        }
        const uint32_t s = ((len + kG * 4u - 1u) / (kG * 4u)) * 4u;     // block bytes, multiple of 4
        const uint32_t pad = kG * s - len;
        // lane's block in the padded frame: [lane*s, (lane+1)*s) -> message bytes [lo, hi)
        const uint32_t fb = lane * s;
        const uint32_t lo = fb > pad ? fb - pad : 0u;
        const uint32_t hi = fb + s > pad ? fb + s - pad : 0u;
        uint32_t c = crc_range(L[0], 0u, p + lo, hi - lo);         // raw: from state 0
        // log2(G) combine levels: lane j with j % 2d == 2d - 1 takes shift(c[j - d], d s) ^ c[j].
        // Strided batches bring the level multipliers x^(8 s 2^k) and x^(8 L) from the host.
        const bool pre = A.lens == nullptr;
        uint32_t xs = pre ? A.xs[0] : x8n(s);
#pragma unroll
        for (int k = 0, d = 1; d < kG; ++k, d <<= 1) {
            const uint32_t left = (uint32_t)__shfl_up((int)c, d, kG);
            if ((lane & (2u * d - 1u)) == 2u * d - 1u) {
                c ^= multmodp(pre ? A.xs[k] : xs, left);
            }
            if (!pre && d < kG / 2) {
                xs = multmodp(xs, xs);
            }
        }
        if (valid && lane == kG - 1) {
            c ^= multmodp(pre ? A.xl : x8n(len), 0xFFFFFFFFu);          // the register's initial value
            A.out[i] = crc_finish(c, len, A.cpl != 0u);
        }
    }
}

}  // namespace

namespace {

// Host twins of multmodp / x8n (the level multipliers of a strided batch are batch constants).
uint32_t h_multmodp(uint32_t a, uint32_t b) {
    uint32_t p = 0u;
    for (int i = 31; i >= 0; --i) {
        p ^= ((a >> i) & 1u) ? b : 0u;
        b = (b & 1u) ? ((b >> 1) ^ kPoly) : (b >> 1);
    }
    return p;
}

uint32_t h_x8n(uint64_t n) {
    uint32_t sq = 0x00800000u;                                   // x^8
    uint32_t p = 0x80000000u;
    for (; n != 0u; n >>= 1) {
        if (n & 1u) p = h_multmodp(sq, p);
        sq = h_multmodp(sq, sq);
    }
    return p;
}

thread_local TuneKnob g_crc_kernel{0};      // NETCSUM_TUNE_CRC_KERNEL (netcsum_mi355x.h)
thread_local TuneKnob g_crc_lanes{0};       // NETCSUM_TUNE_CRC_LANES: interleaved lanes per segment, 0 auto
thread_local TuneKnob g_crc_nt{0};          // NETCSUM_TUNE_CRC_NT: non-temporal chunk loads (interleaved form)
thread_local TuneKnob g_crc_wide{1};        // NETCSUM_TUNE_CRC_WIDE: 0 byte, 1 11-bit, 2 lane-replicated 6-bit tables

enum class CrcForm { Lane, Block, Ilv1, Ilv2, Ilv4, Ilv8, Ilv16 };

CrcForm ilv_form(uint32_t max_len, bool varlen) {
    switch (g_crc_lanes.load()) {
    case 1: return CrcForm::Ilv1;
    case 2: return CrcForm::Ilv2;
    case 4: return CrcForm::Ilv4;
    case 8: return CrcForm::Ilv8;
    case 16: return CrcForm::Ilv16;
    default: return !varlen && max_len >= 1024u ? CrcForm::Ilv8 : CrcForm::Ilv4;   // tools/crc_probe.py sweep
    }
}

CrcForm crc_form(uint32_t max_len, bool varlen) {
    switch (g_crc_kernel.load()) {
    case 1: return max_len <= kCrcShortMax && !varlen ? CrcForm::Lane : CrcForm::Block;
    case 2: return ilv_form(max_len, varlen);
    case 3: return CrcForm::Lane;
    default: return max_len <= kCrcShortMax && !varlen ? CrcForm::Lane : ilv_form(max_len, varlen);
    }
}

}  // namespace

void set_crc_kernel(int v) { g_crc_kernel.store(v); }
void set_crc_lanes(int v) { g_crc_lanes.store(v); }
void set_crc_nt(int v) { g_crc_nt.store(v); }
void set_crc_wide(int v) { g_crc_wide.store(v); }

const char* crc_launch_name(uint32_t max_len, bool varlen) {
    // [table form][nt][log2 G]: "crc_ilv_kernel<nt,w11> G=4 block=512", ...
    static const std::vector<std::string> names = [] {
        std::vector<std::string> v;
        for (int w = 0; w < 3; ++w) {
            for (int nt = 0; nt < 2; ++nt) {
                for (int g = 1; g <= 16; g *= 2) {
                    std::string t = nt ? "nt" : "";
                    if (w != 0) t += std::string(t.empty() ? "" : ",") + (w == 1 ? "w11" : "k6");
                    v.push_back("crc_ilv_kernel" + (t.empty() ? t : "<" + t + ">") + " G=" + std::to_string(g) +
                                " block=" + std::to_string(ilv_block(w)));
                }
            }
        }
        return v;
    }();
    const int w = std::min(std::max(g_crc_wide.load(), 0), 2);
    const int base = 10 * w + (g_crc_nt.load() != 0 ? 5 : 0);
    switch (crc_form(max_len, varlen)) {
    case CrcForm::Lane: return !varlen && max_len <= 16u ? "crc_tiny_kernel block=256" : "crc_lane_kernel block=256";
    case CrcForm::Block: return "crc_group_kernel G=16 block=256";
    case CrcForm::Ilv1: return names[base + 0].c_str();
    case CrcForm::Ilv2: return names[base + 1].c_str();
    case CrcForm::Ilv4: return names[base + 2].c_str();
    case CrcForm::Ilv8: return names[base + 3].c_str();
    default: return names[base + 4].c_str();
    }
}

template <int G, int W>
static void launch_ilv_w(const CrcBatchArgs& a, uint32_t cu, hipStream_t s) {
    constexpr uint32_t B = ilv_block(W);
    const uint32_t steps = (a.n + (B / G) - 1u) / (B / G);
    // blocks resident per CU by LDS: byte tables 24 / 20 / <= 16 KiB (256 threads); W 1 44 .. 60 KiB
    // (512); W 2 85 .. 97 KiB (1024)
    const uint32_t per_cu = W == 2 ? 1u : W == 1 ? (G >= 8 ? 2u : 3u) : (G == 16 ? 6u : G == 8 ? 8u : 10u);
    const uint32_t grid = std::min<uint32_t>(steps, cu * per_cu);
    if (g_crc_nt.load()) {
        hipLaunchKernelGGL((crc_ilv_kernel<G, true, W>), dim3(grid), dim3(B), 0, s, a);
    } else {
        hipLaunchKernelGGL((crc_ilv_kernel<G, false, W>), dim3(grid), dim3(B), 0, s, a);
    }
}

template <int G>
static void launch_ilv(const CrcBatchArgs& a, uint32_t cu, hipStream_t s) {
    switch (g_crc_wide.load()) {
    case 0: launch_ilv_w<G, 0>(a, cu, s); break;
    case 2: launch_ilv_w<G, 2>(a, cu, s); break;
    default: launch_ilv_w<G, 1>(a, cu, s); break;
    }
}

hipError_t launch_crc_batch(const CrcBatchArgs& a0, uint32_t max_len, int cus, hipStream_t s) {
    if (a0.n == 0u) return hipSuccess;
    CrcBatchArgs a = a0;
    const uint32_t cu = (uint32_t)std::max(1, cus);
    const bool varlen = a.lens != nullptr;
    switch (crc_form(max_len, varlen)) {
    case CrcForm::Lane: {
        const uint32_t grid = std::min<uint32_t>((a.n + 255u) / 256u, cu * 8u);   // LDS 4 KiB per block
        if (!varlen && a.off == nullptr && a.len <= 16u) {
            hipLaunchKernelGGL(crc_tiny_kernel, dim3(grid), dim3(256), 0, s, a);
        } else {
            hipLaunchKernelGGL(crc_lane_kernel, dim3(grid), dim3(256), 0, s, a);
        }
        break;
    }
    case CrcForm::Block: {
        if (!varlen) {
            const uint32_t sb = ((a.len + kG * 4u - 1u) / (kG * 4u)) * 4u;
            uint32_t x = h_x8n(sb);
            for (int k = 0; k < 4; ++k) {
                a.xs[k] = x;
                x = h_multmodp(x, x);
            }
            a.xl = h_x8n(a.len);
        }
        const uint32_t steps = (a.n + (256u / kG) - 1u) / (256u / kG);
        hipLaunchKernelGGL(crc_group_kernel, dim3(std::min<uint32_t>(steps, cu * 8u)), dim3(256), 0, s, a);
        break;
    }
    case CrcForm::Ilv1: launch_ilv<1>(a, cu, s); break;
    case CrcForm::Ilv2: launch_ilv<2>(a, cu, s); break;
    case CrcForm::Ilv4: launch_ilv<4>(a, cu, s); break;
    case CrcForm::Ilv8: launch_ilv<8>(a, cu, s); break;
    default: launch_ilv<16>(a, cu, s); break;
    }
    return hipGetLastError();
}

}  // namespace netcsum
