// netcsum_kernels.h — internal interface between the C ABI (netcsum_abi.hip) and the kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace netcsum {

struct SegBatchArgs {
    const uint8_t*  base;          // strided: first segment; varlen: base of the offsets
    const uint64_t* seg_off;       // varlen only (nullptr => strided)
    const uint16_t* seg_len_v;     // varlen only
    uint64_t        seg_stride;    // strided only
    uint32_t        seg_len;       // strided only
    const uint8_t*  pseudo;        // nullptr => no pseudo-header
    uint32_t        pseudo_stride;
    uint32_t        pseudo_len;
    uint32_t        n_seg;
    uint32_t        verify;        // 0: u16 checksum out, 1: u8 DEF_OK/DEF_FAIL out
    void*           out;
};

struct LaunchCfg {
    int  grid;             // workgroups
    int  block;            // threads per workgroup (multiple of 64)
    int  group_lanes;      // lanes per segment: 1, 4, 8, 16, 32, 64
    int  chunks_per_pass;  // 16-B chunks per lane per pass: 1..4
    bool nt;               // non-temporal segment loads
};

hipError_t launch_seg_batch(const SegBatchArgs& a, const LaunchCfg& c, hipStream_t s);
hipError_t launch_stream_exact(const void* d_p, uint32_t n16, unsigned long long* d_sum, int grid,
                               hipStream_t s);
hipError_t launch_fill(void* d_buf, uint64_t n_bytes, uint64_t first_byte, uint64_t seed, int pattern, int grid,
                       hipStream_t s);
hipError_t launch_read_stream(const void* d_p, uint64_t n16, unsigned long long* d_sink, int grid, bool nt,
                              hipStream_t s);

}  // namespace netcsum
