// netcsum_crc.hip — gfx950 CRC-32 of µC/TCP-IP's Source/net_util.c:485-636: the IEEE 802.3
// polynomial in reflected form (0xEDB88320, net_util.c:77), register initialised to 0xFFFFFFFF
// (NET_UTIL_32_BIT_ONES_CPL_NEG_ZERO, :58), octets shifted in LSB first (:510-524);
// NetUtil_32BitCRC_Calc returns the register as is, NetUtil_32BitCRC_CalcCpl complemented (:583).
// The reference's callers hash 6-byte multicast MAC addresses (Dev/Ether/*/net_dev_*.c,
// AddrMulticastAdd / Remove); the batch form here takes any number of segments of any length.
//
// Arithmetic. The register update is linear over GF(2): processing message M from state I gives
// A^|M|(I) xor raw(M), where raw() is the CRC from state 0 and A^n multiplies by x^(8n) modulo the
// polynomial. So
//   * a segment splits into G equal blocks of s bytes (s a multiple of 4) after a front pad of
//     P = G*s - L zero octets — leading zeros leave raw() unchanged — and lane j of a G-lane group
//     computes raw(block j) with 4-KiB slicing-by-4 tables in LDS;
//   * the group combines the blocks in log2(G) shuffle levels, level k merging pairs at distance
//     2^k with the fixed multiplier x^(8 s 2^k) (squared from level to level);
//   * the initial 0xFFFFFFFF contributes x^(8L) * 0xFFFFFFFF, added once per segment.
// Powers x^(8n) come from the 32 squares x^(2^k) (kX2n) by square-and-multiply, as in zlib's
// crc32_combine. Segments up to kShortMax bytes take one lane each (G = 1: register from
// 0xFFFFFFFF, no combine).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "netcsum_device.h"
#include "netcsum_kernels.h"

namespace netcsum {

namespace {

constexpr uint32_t kPoly = 0xEDB88320u;

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

struct CrcTables {
    uint32_t t[4][256];
};

// T0 = the byte table of net_util.c:512-521's bit loop; T1..T3 = slicing-by-4 tables.
__device__ __forceinline__ void build_tables(CrcTables& T) {
    const uint32_t i = threadIdx.x;                             // blockDim.x == 256
    uint32_t c = i;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        c = (c & 1u) ? ((c >> 1) ^ kPoly) : (c >> 1);
    }
    T.t[0][i] = c;
    __syncthreads();
#pragma unroll
    for (int k = 1; k < 4; ++k) {
        const uint32_t v = T.t[k - 1][i];
        T.t[k][i] = (v >> 8) ^ T.t[0][v & 0xFFu];
        __syncthreads();
    }
}

__device__ __forceinline__ uint32_t crc_byte(const CrcTables& T, uint32_t c, uint32_t b) {
    return T.t[0][(c ^ b) & 0xFFu] ^ (c >> 8);
}

__device__ __forceinline__ uint32_t crc_word(const CrcTables& T, uint32_t c, uint32_t w) {   // 4 octets, LE
    c ^= w;
    return T.t[3][c & 0xFFu] ^ T.t[2][(c >> 8) & 0xFFu] ^ T.t[1][(c >> 16) & 0xFFu] ^ T.t[0][c >> 24];
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

__device__ __forceinline__ uint32_t crc_16(const CrcTables& T, uint32_t c, const uint4& a, const uint4& b, uint32_t sh) {
    c = crc_word(T, c, win16_dword(a, b, sh, 0));
    c = crc_word(T, c, win16_dword(a, b, sh, 1));
    c = crc_word(T, c, win16_dword(a, b, sh, 2));
    return crc_word(T, c, win16_dword(a, b, sh, 3));
}

// Register c advanced over bytes [p, p + n): whole ALIGNED 16-B loads (a chunk holding any byte of
// the range lies in the range's pages, so reading all of it cannot fault), 64 B of the range per
// step from five loads issued together, the stream's dwords cut out by v_alignbyte_b32; the last
// n mod 4 octets one at a time. (A per-byte head loop with a load per octet made the lanes wait on
// one dependent load after another: 1.75 ms for 1 M x 1500 B.)
__device__ uint32_t crc_range(const CrcTables& T, uint32_t c, const uint8_t* p, uint32_t n) {
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
    const uint8_t* t = p + done;
    for (; done < n; ++done) {
        c = crc_byte(T, c, *t++);
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
// built once per block, which then walks its share of the batch 256 segments at a time.
__global__ void __launch_bounds__(256) crc_lane_kernel(CrcBatchArgs A) {
    __shared__ CrcTables T;
    build_tables(T);
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < A.n; i += gridDim.x * 256u) {
        const uint8_t* p;
        uint32_t len;
        seg_desc(A, i, p, len);
        A.out[i] = crc_finish(crc_range(T, 0xFFFFFFFFu, p, len), len, A.cpl != 0u);
    }
}

// A 16-lane group per segment (4 segments per wave, 16 per block and step), persistent blocks.
constexpr int kG = 16;

__global__ void __launch_bounds__(256) crc_group_kernel(CrcBatchArgs A) {
    __shared__ CrcTables T;
    build_tables(T);
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
        uint32_t c = crc_range(T, 0u, p + lo, hi - lo);                // raw: from state 0
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

}  // namespace

hipError_t launch_crc_batch(const CrcBatchArgs& a0, uint32_t max_len, int cus, hipStream_t s) {
    if (a0.n == 0u) return hipSuccess;
    CrcBatchArgs a = a0;
    const uint32_t resident = (uint32_t)std::max(1, cus) * 8u;        // blocks that fit at once (LDS 4 KiB each)
    if (max_len <= kCrcShortMax) {
        const uint32_t grid = std::min<uint32_t>((a.n + 255u) / 256u, resident);
        hipLaunchKernelGGL(crc_lane_kernel, dim3(grid), dim3(256), 0, s, a);
    } else {
        if (a.lens == nullptr) {
            const uint32_t sb = ((a.len + kG * 4u - 1u) / (kG * 4u)) * 4u;
            uint32_t x = h_x8n(sb);
            for (int k = 0; k < 4; ++k) {
                a.xs[k] = x;
                x = h_multmodp(x, x);
            }
            a.xl = h_x8n(a.len);
        }
        const uint32_t steps = (a.n + (256u / kG) - 1u) / (256u / kG);
        const uint32_t grid = std::min<uint32_t>(steps, resident);
        hipLaunchKernelGGL(crc_group_kernel, dim3(grid), dim3(256), 0, s, a);
    }
    return hipGetLastError();
}

}  // namespace netcsum
