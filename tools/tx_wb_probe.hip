// Tx write-back probe (not product code): what does writing the two checksum fields of 1 M packed
// 1500-B datagrams cost, by write form, once the dirty lines reach HBM?
//
// Each variant W runs as "W, then a read stream over the same 1.5 GB" (the next Tx launch reads the
// batch again), timed with events over 20 pairs; the cost of W is pair - (read stream alone).
//   field2      two 2-B stores per datagram at +10 and +36 (what pkt_scatter_kernel does)
//   sector64    the aligned 64-B sector(s) holding the fields rewritten whole (16-B stores, 4 lanes)
//   line128     the aligned 128-B line(s) holding the fields rewritten whole (16-B stores, 8 lanes)
//   load_field2 a plain 16-B load of the field's line first (line allocated valid in L2), then field2
//   dense8      one 8-B record per datagram into a dense array (the lower bound of any write)
//   sector32    the aligned 32-B sector(s) holding the fields rewritten whole (16-B stores, 2 lanes)
//   load_sector32  the same sectors loaded first (plain), the field patched, the sectors written whole
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/build/tx_wb_probe tools/tx_wb_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                 \
        }                                                                                 \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void fill_kernel(u32x4* p, uint64_t n16) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) {
        uint32_t x = (uint32_t)i * 2654435761u;
        p[i] = u32x4{x, x ^ 0x9E3779B9u, x + 7u, ~x};
    }
}

__global__ void read_kernel(const u32x4* p, uint64_t n16, uint32_t* sink) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) {
        u32x4 v = __builtin_nontemporal_load(p + i);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) {
        sink[0] = acc;
    }
}

__global__ void field2_kernel(uint8_t* base, uint32_t n, uint32_t stride, uint32_t salt) {
    uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) {
        uint8_t* p = base + (uint64_t)i * stride;
        *(uint16_t*)(p + 10) = (uint16_t)(i ^ salt);
        *(uint16_t*)(p + 36) = (uint16_t)(i + salt);
    }
}

__global__ void load_field2_kernel(uint8_t* base, uint32_t n, uint32_t stride, uint32_t salt) {
    uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) {
        uint8_t* p = base + (uint64_t)i * stride;
        const u32x4* a = (const u32x4*)((uintptr_t)(p + 10) & ~(uintptr_t)15);
        const u32x4* b = (const u32x4*)((uintptr_t)(p + 36) & ~(uintptr_t)15);
        u32x4 va = *a, vb = *b;
        *(uint16_t*)(p + 10) = (uint16_t)(va.x ^ salt);
        *(uint16_t*)(p + 36) = (uint16_t)(vb.y + salt);
    }
}

// G lanes per datagram rewrite the aligned G*16-B block(s) holding +10 and +36 (G = 2: 32 B, 4: 64 B, 8: 128 B)
template <int G>
__global__ void block_kernel(uint8_t* base, uint32_t n, uint32_t stride, uint32_t salt) {
    uint32_t t = blockIdx.x * 256 + threadIdx.x;
    uint32_t i = t / G, l = t % G;
    if (i < n) {
        uintptr_t p = (uintptr_t)base + (uint64_t)i * stride;
        uintptr_t b0 = (p + 10) & ~(uintptr_t)(G * 16 - 1);
        uintptr_t b1 = (p + 37) & ~(uintptr_t)(G * 16 - 1);
        u32x4 v = u32x4{i, salt, i ^ salt, l};
        *(u32x4*)(b0 + 16 * l) = v;
        if (b1 != b0) {
            *(u32x4*)(b1 + 16 * l) = v;
        }
    }
}

// 2 lanes per datagram: each loads its 16 B of the 32-B sector(s) holding the fields and writes them back
__global__ void load_sector32_kernel(uint8_t* base, uint32_t n, uint32_t stride, uint32_t salt) {
    uint32_t t = blockIdx.x * 256 + threadIdx.x;
    uint32_t i = t / 2, l = t % 2;
    if (i < n) {
        uintptr_t p = (uintptr_t)base + (uint64_t)i * stride;
        uintptr_t b0 = (p + 10) & ~(uintptr_t)31;
        uintptr_t b1 = (p + 37) & ~(uintptr_t)31;
        u32x4 v0 = *(const u32x4*)(b0 + 16 * l);
        u32x4 v1 = b1 != b0 ? *(const u32x4*)(b1 + 16 * l) : v0;
        v0.x ^= salt;
        v1.y ^= salt;
        *(u32x4*)(b0 + 16 * l) = v0;
        if (b1 != b0) {
            *(u32x4*)(b1 + 16 * l) = v1;
        }
    }
}

__global__ void dense8_kernel(uint64_t* rec, uint32_t n, uint32_t salt) {
    uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) {
        rec[i] = ((uint64_t)i << 32) | salt;
    }
}

int main(int argc, char** argv) {
    const uint32_t n = 1u << 20, stride = argc > 1 ? (uint32_t)std::atoi(argv[1]) : 1500u;
    const uint64_t bytes = (uint64_t)n * stride + 256, n16 = bytes / 16;
    uint8_t* buf;
    uint64_t* rec;
    uint32_t* sink;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&rec, (uint64_t)n * 8));
    CK(hipMalloc(&sink, 64));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, s, (u32x4*)buf, n16);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const uint32_t rgrid = 256 * 32;
    auto rd = [&]() { hipLaunchKernelGGL(read_kernel, dim3(rgrid), dim3(256), 0, s, (const u32x4*)buf, n16, sink); };
    auto wr = [&](int v, uint32_t salt) {
        switch (v) {
        case 0: break;
        case 1: hipLaunchKernelGGL(field2_kernel, dim3((n + 255) / 256), dim3(256), 0, s, buf, n, stride, salt); break;
        case 2: hipLaunchKernelGGL(block_kernel<4>, dim3((4 * n + 255) / 256), dim3(256), 0, s, buf, n, stride, salt); break;
        case 3: hipLaunchKernelGGL(block_kernel<8>, dim3((8 * n + 255) / 256), dim3(256), 0, s, buf, n, stride, salt); break;
        case 4: hipLaunchKernelGGL(load_field2_kernel, dim3((n + 255) / 256), dim3(256), 0, s, buf, n, stride, salt); break;
        case 5: hipLaunchKernelGGL(dense8_kernel, dim3((n + 255) / 256), dim3(256), 0, s, rec, n, salt); break;
        case 6: hipLaunchKernelGGL(block_kernel<2>, dim3((2 * n + 255) / 256), dim3(256), 0, s, buf, n, stride, salt); break;
        case 7: hipLaunchKernelGGL(load_sector32_kernel, dim3((2 * n + 255) / 256), dim3(256), 0, s, buf, n, stride, salt); break;
        }
    };
    const char* names[] = {"read_only", "field2", "sector64", "line128", "load_field2", "dense8", "sector32", "load_sector32"};
    const int reps = 20;
    for (int pass = 0; pass < 2; ++pass) {
        for (int v = 0; v < 8; ++v) {
            for (int k = 0; k < 30; ++k) {      // warm clocks and caches
                wr(v, k);
                rd();
            }
            CK(hipStreamSynchronize(s));
            // the pair
            CK(hipEventRecord(e0, s));
            for (int k = 0; k < reps; ++k) {
                wr(v, k);
                rd();
            }
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms_pair;
            CK(hipEventElapsedTime(&ms_pair, e0, e1));
            // the write kernel alone (its own duration, before its write-back)
            float ms_w = 0.f;
            if (v) {
                for (int k = 0; k < reps; ++k) {
                    rd();
                    CK(hipEventRecord(e0, s));
                    wr(v, k);
                    CK(hipEventRecord(e1, s));
                    CK(hipEventSynchronize(e1));
                    float t;
                    CK(hipEventElapsedTime(&t, e0, e1));
                    ms_w += t;
                }
            }
            std::printf("{\"pass\": %d, \"stride\": %u, \"variant\": \"%s\", \"ms_pair\": %.4f, \"ms_write_kernel\": %.4f}\n",
                        pass, stride, names[v], ms_pair / reps, ms_w / reps);
            std::fflush(stdout);
        }
    }
    CK(hipStreamSynchronize(s));
    return 0;
}
