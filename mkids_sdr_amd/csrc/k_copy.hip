// Stream-copy probe (bench.py's measured HBM roof, SURVEY.md §8(d) "report against a measured
// stream-copy peak in the same run"): dst = src. Not on the hot path.
#include "mkid_internal.h"

namespace mkid {

// The plain float4 copy (one 16-byte load + store per thread, one thread per 16 bytes): the form
// MI355X_MICROARCH.md quotes its measured 6.29 TB/s for.
__global__ __launch_bounds__(256) void k_stream_copy(uint4* __restrict__ dst, const uint4* __restrict__ src,
                                                     int64_t n16) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n16) dst[i] = src[i];
}

hipError_t launch_stream_copy(void* dst, const void* src, int64_t bytes, hipStream_t s) {
    const int64_t n16 = bytes / 16;
    if (n16 <= 0) return hipSuccess;
    const int64_t blocks = (n16 + 255) / 256;
    if (blocks > 0x7fffffff) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_stream_copy, dim3((unsigned)blocks), dim3(256), 0, s, (uint4*)dst, (const uint4*)src, n16);
    return hipGetLastError();
}

}  // namespace mkid
