// Stream-copy probe (bench.py's measured HBM roof, SURVEY.md §8(d) "report against a measured
// stream-copy peak in the same run"): dst = src, 16 B per lane per access, non-temporal both
// ways, grid-stride over a grid sized to fill every CU several times. Not on the hot path.
#include "mkid_internal.h"

namespace mkid {

__global__ __launch_bounds__(256) void k_stream_copy(uint4* __restrict__ dst, const uint4* __restrict__ src,
                                                     int64_t n16) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const int64_t stride = (int64_t)gridDim.x * 256 * 4;
    for (int64_t i = (int64_t)blockIdx.x * 256 * 4 + threadIdx.x; i < n16; i += stride) {
        u32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (i + u * 256 < n16) v[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src) + i + u * 256);
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (i + u * 256 < n16) __builtin_nontemporal_store(v[u], reinterpret_cast<u32x4*>(dst) + i + u * 256);
    }
}

hipError_t launch_stream_copy(void* dst, const void* src, int64_t bytes, hipStream_t s) {
    const int64_t n16 = bytes / 16;
    if (n16 <= 0) return hipSuccess;
    int64_t blocks = (n16 + 1023) / 1024;
    if (blocks > 256 * 16) blocks = 256 * 16;
    hipLaunchKernelGGL(k_stream_copy, dim3((unsigned)blocks), dim3(256), 0, s, (uint4*)dst, (const uint4*)src, n16);
    return hipGetLastError();
}

}  // namespace mkid
