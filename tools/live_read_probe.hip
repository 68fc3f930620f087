// Live-sector read probe (not product code): how fast can the run-stream access pattern read only the
// 64-B sectors that hold datagram bytes of a strided NIC ring, with nothing computed? The floor of
// the packet run-stream kernel's live-piece forms (DESIGN §9 "NIC-ring layouts").
//
// Ring: n slots of `stride` bytes, each holding `len` datagram bytes at +lead. A wave owns a run of R
// slots and reads it as 1-KiB pieces from the 128-B line below the run (lane l: 16 B at 16 l), D = 4
// pieces in flight, nt loads — as pkt_stream_kernel does — in one of two forms:
//   whole  every piece of the run's span (the kernel's bound 0)
//   live   only pieces holding a live sector, each lane loading its 16 B only if its sector is live
//          (the kernel's bounds 1-3; the sector bitmap is precomputed here, one bit per 64-B sector
//          of the ring, 1/512 of the ring's bytes, read once per run)
// with D = 4 or 8 pieces in flight, and optionally ".touch": before the stream, lane k loads the 16 B
// at datagram k's start with the plain policy (what the kernel's header parse does, and what the
// row touch of DESIGN §5.2 does for the segment kernels)
// and only adds the loaded words up. Median of 20 HIP-event timed launches after a warm-up, per
// (layout, form, R); one JSON line each: ms, datagram GB/s, fraction of 8 TB/s, sector bytes.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/build/live_read_probe tools/live_read_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                 \
        }                                                                                 \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t kOOB = 0x80000000u;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ u32x4 ld16(__amdgpu_buffer_rsrc_t r, uint32_t voff) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, 0, 2);
}

__device__ __forceinline__ u32x4 opaque(u32x4 v) {
    asm volatile("" : "+v"(v));
    return v;
}

__device__ __forceinline__ uint32_t add4(u32x4 v, uint32_t a) {
    return __builtin_amdgcn_sad_u16(v.x, 0u, __builtin_amdgcn_sad_u16(v.y, 0u, __builtin_amdgcn_sad_u16(v.z, 0u, __builtin_amdgcn_sad_u16(v.w, 0u, a))));
}

__global__ void fill_kernel(u32x4* p, uint64_t n16) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) {
        const uint32_t x = (uint32_t)i * 2654435761u;
        p[i] = u32x4{x, x ^ 0x9E3779B9u, x + 7u, ~x};
    }
}

// bit s of bits: sector s (bytes [64 s, 64 s + 64) of the ring) holds datagram bytes (slot i's length:
// lens[i], or `len` for every slot when lens is null); win > 0: a datagram that ends within win bytes of
// its first 16-B chunk holds none (the kernels sum it from the window loaded at its start)
__global__ void sectors_kernel(uint32_t* bits, uint64_t nsect, uint64_t stride, uint32_t lead, uint32_t len,
                               const uint16_t* lens, uint32_t n, uint32_t win) {
    const uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (w * 32u >= nsect) return;
    uint32_t m = 0;
    for (uint32_t b = 0; b < 32u; ++b) {
        const uint64_t s0 = (w * 32u + b) * 64u, s1 = s0 + 64u;
        const uint64_t a = s0 / stride;
        bool live = false;
        for (uint64_t i = a; i <= (s1 - 1u) / stride; ++i) {
            const uint32_t l = lens ? (i < n ? lens[i] : 0u) : len;
            const uint64_t d0 = i * stride + lead, d1 = d0 + l;
            const bool inwin = win != 0u && (uint32_t)(d0 & 15u) + l <= win;
            live = live || (!inwin && s0 < d1 && d0 < s1);
        }
        m |= live ? (1u << b) : 0u;
    }
    bits[w] = m;
}

__device__ __forceinline__ uint32_t incl_scan64(uint32_t v, uint32_t lane) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);
    const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)v, 15);
    const uint32_t r1 = (uint32_t)__builtin_amdgcn_readlane((int)v, 31);
    const uint32_t r2 = (uint32_t)__builtin_amdgcn_readlane((int)v, 47);
    return v + (lane >= 16u ? r0 : 0u) + (lane >= 32u ? r1 : 0u) + (lane >= 48u ? r2 : 0u);
}

// LIVE: 0 every piece of the span, 1 the live pieces (lanes load their live sectors), 2 the live
// sectors compacted (16 per wave-instruction, in address order: lane l the 16 B at (l & 3) 16 of live
// sector 16 q + l / 4). TOUCH: 0 none, 1 lane k loads the 16 B at datagram k's start (plain), 2 the six
// 16-B chunks from there (the packet kernels' 96-B header window).
template <int LIVE, int D, int TOUCH>
__global__ void __launch_bounds__(256) probe_kernel(const uint8_t* ring, uint64_t ring_bytes, uint32_t n, uint64_t stride,
                                                    uint32_t lead, uint32_t len, uint32_t R, const uint32_t* bits,
                                                    uint32_t* sink) {
    __shared__ uint16_t lst_all[4][1024];
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t s_begin = ((uint64_t)blockIdx.x * 4u + w) * R;
    if (s_begin >= n) return;
    const uint32_t nres = (uint32_t)std::min<uint64_t>(R, n - s_begin);
    const uint64_t a0 = s_begin * stride + lead;                       // the run's first datagram byte
    const uint64_t O = a0 & ~127ull;
    const uint32_t span = (uint32_t)(a0 - O) + (uint32_t)((nres - 1u) * stride) + len;
    const uint32_t npieces = (span + 1023u) >> 10;
    const __amdgpu_buffer_rsrc_t rd = rsrc(ring + O, (span + 15u) & ~15u);
    const uint32_t lane16 = 16u * lane;
    uint64_t lm = 0;                                                     // live pieces (bit 63: sentinel)
    uint32_t pm = 0;                                                     // sector mask of piece `lane`
    if constexpr (LIVE != 0) {
        // piece `lane`: its 16 sectors start at sector O / 64 + 16 lane (O is 128-B aligned)
        const uint64_t s = O / 64u + 16u * lane;
        if (lane < npieces) {                                            // (words inside the bitmap)
            const uint32_t lo = bits[s >> 5], hi = bits[(s >> 5) + 1u];
            pm = (uint32_t)((((uint64_t)hi << 32) | lo) >> (s & 31u)) & 0xFFFFu;
        }
        lm = __builtin_amdgcn_ballot_w64(pm != 0u) | (1ull << 63);
    }
    const uint32_t lbit = 1u << (lane >> 2);
    uint32_t nsect = 0;
    uint16_t* lst = lst_all[w];
    if constexpr (LIVE == 2) {
        const uint32_t cnt = (uint32_t)__builtin_popcount(pm);
        const uint32_t incl = incl_scan64(cnt, lane);
        nsect = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        for (uint32_t m = pm, pos = incl - cnt; m != 0u; m &= m - 1u) lst[pos++] = (uint16_t)((lane << 4) | (uint32_t)__builtin_ctz(m));
        __builtin_amdgcn_wave_barrier();
    }
    auto pop = [&]() -> uint32_t {
        const uint32_t q = (uint32_t)__builtin_ctzll(lm);
        lm = (lm & (lm - 1u)) | (1ull << 63);
        return q;
    };
    auto voff = [&](uint32_t q) -> uint32_t {
        if constexpr (LIVE == 2) {
            const uint32_t i = (q << 4) + (lane >> 2);
            return i < nsect ? ((uint32_t)lst[i < 1023u ? i : 1023u] << 6) + ((lane & 3u) << 4) : kOOB;
        } else {
            const uint32_t sm = (uint32_t)__builtin_amdgcn_readlane((int)pm, (int)q);
            return (sm & lbit) ? (q << 10) + lane16 : kOOB;
        }
    };
    const uint32_t nlive = LIVE == 2 ? (nsect + 15u) >> 4 : LIVE ? (uint32_t)__builtin_popcountll(lm) - 1u : npieces;
    // touch: lane k loads the 16 B at datagram k's start (plain policy), as the kernel's parse does; TOUCH
    // 2: the 96-B header window (six chunks)
    u32x4 tv = {0u, 0u, 0u, 0u};
    if constexpr (TOUCH != 0) {
        const uint32_t t0 = lane < nres ? ((uint32_t)(a0 - O) + lane * (uint32_t)stride) & ~15u : kOOB;
#pragma unroll
        for (int c = 0; c < (TOUCH == 2 ? 6 : 1); ++c) {
            const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rd, (int)(t0 == kOOB ? kOOB : t0 + 16u * (uint32_t)c), 0, 0);
            tv = u32x4{tv.x ^ x.x, tv.y ^ x.y, tv.z ^ x.z, tv.w ^ x.w};
        }
    }
    u32x4 dv[D];
    uint32_t qd[D];
#pragma unroll
    for (int j = 0; j < D; ++j) {
        qd[j] = LIVE == 1 ? pop() : (uint32_t)j;
        dv[j] = ld16(rd, LIVE ? voff(qd[j]) : ((uint32_t)j << 10) + lane16);
    }
    uint32_t acc = 0;
    const uint32_t rounds = (nlive + D - 1u) / D;
    for (uint32_t r = 0; r < rounds; ++r) {
#pragma unroll
        for (int j = 0; j < D; ++j) {
            acc = add4(opaque(dv[j]), acc);
            if constexpr (LIVE == 1) {
                qd[j] = pop();
                dv[j] = ld16(rd, voff(qd[j]));
            } else if constexpr (LIVE == 2) {
                qd[j] += (uint32_t)D;
                dv[j] = ld16(rd, voff(qd[j]));
            } else {
                dv[j] = ld16(rd, ((r * D + (uint32_t)j + D) << 10) + lane16);
            }
            asm volatile("" ::: "memory");
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    acc = add4(tv, acc);
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

int main(int argc, char** argv) {
    struct Layout {
        const char* name;
        uint64_t stride;
        uint32_t lead, len;
        int mix;           // 0 uniform `len`; 1 segments 20 / 556 / 1480 B; 2 datagrams 40 / 576 / 1500 B (7 : 4 : 1)
        uint32_t win;      // sectors of datagrams ending within `win` B of their first chunk are not live
    };
    // default: the packet rows' rings; or layouts from the command line as NAME STRIDE LEAD LEN ...
    // (round 5: TCP segments at TransportHdrIx of pool buffers, `seg1520 1520 34 1480`, `seg2k 2048 84
    // 1480`, and the chain row's fragments, `frag2k 2048 42 1480`; LEN `mix`: segments of 20 / 556 /
    // 1480 B at 7 : 4 : 1 — the 40 / 576 / 1500-B datagram mix — drawn per slot, `seg1520mix 1520 34 mix`)
    // (round 6: LEN `mixwin`: the segment mix with the pool kernel's in-window rule — a segment ending
    // within 48 B of its first chunk is read by that lane's window loads, not as sectors; `ringmix`: the
    // 40 / 576 / 1500-B datagram mix with the packet kernel's 96-B header window, `ring 1520 14 ringmix`)
    std::vector<Layout> layouts = {{"packed", 1500, 0, 1500, 0, 0}, {"template", 1520, 14, 1500, 0, 0},
                                   {"nb2k", 2048, 64, 1500, 0, 0}};
    if (argc > 1) {
        layouts.clear();
        for (int i = 1; i + 3 < argc; i += 4) {
            const uint64_t st = std::strtoull(argv[i + 1], nullptr, 10);
            const std::string lt = argv[i + 3];
            const int mix = (lt == "mix" || lt == "mixwin") ? 1 : lt == "ringmix" ? 2 : 0;
            const uint32_t win = lt == "mixwin" ? 48u : lt == "ringmix" ? 96u : 0u;
            const uint32_t ld = (uint32_t)std::strtoul(argv[i + 2], nullptr, 10),
                           ln = mix == 1 ? 1480u : mix == 2 ? 1500u : (uint32_t)std::strtoul(argv[i + 3], nullptr, 10);
            if (st == 0 || st > 2048u || ld + ln > st) {
                std::fprintf(stderr, "layout %s: need stride <= 2048 and lead + len <= stride\n", argv[i]);
                return 2;
            }
            layouts.push_back({argv[i], st, ld, ln, mix, win});
        }
    }
    const uint32_t n = 1u << 20;
    const uint64_t ring_bytes = (uint64_t)n * 2048u + 4096u;
    uint8_t* ring = nullptr;
    uint32_t *bits = nullptr, *sink = nullptr;
    uint16_t* dlens = nullptr;
    std::vector<uint16_t> hmix(n), hring(n);
    {
        uint64_t x = 0x5EED0001ull;                                      // 20 / 556 / 1480 B at 7 : 4 : 1
        for (uint32_t i = 0; i < n; ++i) {
            x = x * 6364136223846793005ull + 1442695040888963407ull;
            const uint32_t r = (uint32_t)(x >> 33) % 12u;
            hmix[i] = r < 7u ? 20u : r < 11u ? 556u : 1480u;
            hring[i] = (uint16_t)(hmix[i] + 20u);                        // the datagrams: 40 / 576 / 1500 B
        }
    }
    uint16_t* dring = nullptr;
    CK(hipMalloc(&dlens, (size_t)n * 2u));
    CK(hipMemcpy(dlens, hmix.data(), (size_t)n * 2u, hipMemcpyHostToDevice));
    CK(hipMalloc(&dring, (size_t)n * 2u));
    CK(hipMemcpy(dring, hring.data(), (size_t)n * 2u, hipMemcpyHostToDevice));
    CK(hipMalloc(&ring, ring_bytes));
    CK(hipMalloc(&bits, ring_bytes / 64u / 8u + 1024u));
    CK(hipMemset(bits, 0, ring_bytes / 64u / 8u + 1024u));
    CK(hipMalloc(&sink, 64));
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, reinterpret_cast<u32x4*>(ring), ring_bytes / 16u);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (const Layout& L : layouts) {
        const uint64_t bytes = (uint64_t)n * L.stride + 4096u;
        const uint64_t nsect = bytes / 64u;
        const uint16_t* lensp = L.mix == 1 ? dlens : L.mix == 2 ? dring : nullptr;
        hipLaunchKernelGGL(sectors_kernel, dim3((unsigned)((nsect / 32u + 256u) / 256u)), dim3(256), 0, 0, bits, nsect,
                           L.stride, L.lead, L.len, lensp, n, L.win);
        uint64_t dbytes = (uint64_t)n * L.len;
        if (L.mix) {
            dbytes = 0;
            for (uint16_t m : (L.mix == 1 ? hmix : hring)) dbytes += m;
        }
        CK(hipDeviceSynchronize());
        std::vector<uint32_t> hb(nsect / 32u);
        CK(hipMemcpy(hb.data(), bits, hb.size() * 4u, hipMemcpyDeviceToHost));
        uint64_t live = 0;
        for (uint32_t x : hb) live += (uint64_t)__builtin_popcount(x);
        // (form, D, touch): whole / live with 4 pieces in flight, live with the datagram-start touch,
        // live with 8 in flight, with and without the touch
        struct V {
            const char* tag;
            int live, d, touch;
        } vs[] = {{"whole", 0, 4, 0}, {"live", 1, 4, 0}, {"live.touch", 1, 4, 1}, {"live.d8", 1, 8, 0},
                  {"live.d8.touch", 1, 8, 1}, {"whole.touch", 0, 4, 1}, {"compact", 2, 4, 0}, {"compact.touch", 2, 4, 1},
                  {"compact.d8.touch", 2, 8, 1}, {"live.win", 1, 4, 2}, {"compact.win", 2, 4, 2}};
        // (LRP_FORM / LRP_RUN: one form / run length only; LRP_WARM, LRP_PASSES: fewer launches — for
        // a rocprofv3 --pmc pass over one variant)
        const char* only_form = std::getenv("LRP_FORM");
        const uint32_t only_run = std::getenv("LRP_RUN") ? (uint32_t)std::atoi(std::getenv("LRP_RUN")) : 0u;
        const int warm = std::getenv("LRP_WARM") ? std::atoi(std::getenv("LRP_WARM")) : 200;
        const int passes = std::getenv("LRP_PASSES") ? std::atoi(std::getenv("LRP_PASSES")) : 2;
        for (int pass = 0; pass < passes; ++pass) {
            for (const V& v : vs) {
                if ((v.touch == 2) != (L.mix == 2)) continue;            // the 96-B window: the ring only
                if (only_form && std::string(only_form) != v.tag) continue;
                for (uint32_t R : {8u, 16u, 30u, 32u, 41u}) {
                    if (only_run && R != only_run) continue;
                    if ((uint64_t)R * L.stride + 2048u > (63u << 10)) continue;   // a run within the bitmap's reach
                    if ((R == 30u || R == 41u) && (uint64_t)(R + 1u) * L.stride + 2048u <= (63u << 10)) continue;   // (the longest run only)
                    const uint64_t waves = (n + R - 1u) / R;
                    const dim3 g((unsigned)((waves + 3u) / 4u)), b(256);
                    auto launch = [&]() {
#define LRP_L(LV, DD, TT) hipLaunchKernelGGL((probe_kernel<LV, DD, TT>), g, b, 0, 0, ring, bytes, n, L.stride, L.lead, L.len, R, bits, sink)
#define LRP_T(LV, DD) if (v.touch == 0) LRP_L(LV, DD, 0); else if (v.touch == 1) LRP_L(LV, DD, 1); else LRP_L(LV, DD, 2);
                        if (v.live == 0) { LRP_T(0, 4) }
                        else if (v.live == 1 && v.d == 4) { LRP_T(1, 4) }
                        else if (v.live == 1) { LRP_T(1, 8) }
                        else if (v.d == 4) { LRP_T(2, 4) }
                        else { LRP_T(2, 8) }
#undef LRP_T
#undef LRP_L
                    };
                    for (int i = 0; i < warm; ++i) launch();
                    std::vector<float> t(20);
                    for (float& x : t) {
                        CK(hipEventRecord(e0, 0));
                        launch();
                        CK(hipEventRecord(e1, 0));
                        CK(hipEventSynchronize(e1));
                        CK(hipEventElapsedTime(&x, e0, e1));
                    }
                    CK(hipGetLastError());
                    std::sort(t.begin(), t.end());
                    const double ms = t[10], dgram = (double)dbytes;
                    std::printf("{\"layout\": \"%s\", \"stride\": %llu, \"lead\": %u, \"len\": %u, \"form\": \"%s\", \"run\": %u, "
                                "\"pass\": %d, \"ms\": %.4f, \"datagram_GBps\": %.1f, \"frac_of_8TBps\": %.4f, "
                                "\"sector_bytes\": %llu, \"sector_GBps\": %.1f}\n",
                                L.name, (unsigned long long)L.stride, L.lead, L.mix ? 0u : L.len, v.tag, R, pass, ms,
                                dgram / ms / 1e6, dgram / ms / 1e6 / 8000.0, (unsigned long long)(live * 64u),
                                (v.live ? (double)live * 64.0 : (double)n * L.stride) / ms / 1e6);
                    std::fflush(stdout);
                }
            }
        }
    }
    CK(hipFree(ring));
    CK(hipFree(bits));
    CK(hipFree(sink));
    CK(hipFree(dlens));
    CK(hipFree(dring));
    return 0;
}
