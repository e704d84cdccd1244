// Packet compaction (exclusive scan over (channel, segment) counts) and stream-history rolls.
#include "mkid_internal.h"

namespace mkid {

// ---- compaction: exclusive scan of (channel, segment) counts (one block), then copy ----------
constexpr int kScanThreads = 1024;

// d_counts[0] accumulates packets produced, d_counts[1] packets stored in `out` (<= cap), over
// the sub-chunks of one process call (zeroed by the caller at the start of the call).
__global__ __launch_bounds__(kScanThreads) void k_scan_counts(const int32_t* counts, int64_t n_ent,
                                                              int32_t capseg, int64_t cap,
                                                              int64_t* offs, int64_t* d_counts) {
    __shared__ int64_t part[kScanThreads];
    __shared__ unsigned long long tot;
    const int64_t prev = d_counts[1];
    const int64_t per = (n_ent + kScanThreads - 1) / kScanThreads;
    const int64_t b = threadIdx.x * per;
    int64_t sum = 0, sumw = 0;
    for (int64_t i = 0; i < per; ++i)
        if (b + i < n_ent) { const int v = counts[b + i]; sum += v; sumw += v < capseg ? v : capseg; }
    part[threadIdx.x] = sumw;
    if (threadIdx.x == 0) tot = 0;
    __syncthreads();
    for (int off = 1; off < kScanThreads; off <<= 1) {  // Hillis-Steele inclusive scan
        const int64_t v = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    int64_t run = prev + part[threadIdx.x] - sumw;
    for (int64_t i = 0; i < per; ++i)
        if (b + i < n_ent) { offs[b + i] = run; const int v = counts[b + i]; run += v < capseg ? v : capseg; }
    atomicAdd(&tot, (unsigned long long)sum);
    __syncthreads();
    if (threadIdx.x == 0) {
        d_counts[0] += (int64_t)tot;
        const int64_t w = prev + part[kScanThreads - 1];
        d_counts[1] = w < cap ? w : cap;
    }
}

__global__ __launch_bounds__(256) void k_gather_events(const uint64_t* slots, const int32_t* counts,
                                                       int64_t n_ent, int32_t capseg,
                                                       const int64_t* offs, uint64_t* out,
                                                       int64_t cap) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n_ent) return;
    const int n = counts[e] < capseg ? counts[e] : capseg;
    const int64_t o = offs[e];
    for (int i = 0; i < n; ++i)
        if (o + i < cap) out[o + i] = slots[e * capseg + i];
}

hipError_t launch_compact(const uint64_t* slots, const int32_t* counts, int64_t n_ent,
                          int32_t capseg, uint64_t* out, int64_t cap, int64_t* d_counts,
                          int64_t* scan_ws, hipStream_t s) {
    hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(kScanThreads), 0, s, counts, n_ent, capseg,
                       cap, scan_ws, d_counts);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_gather_events, dim3((unsigned)((n_ent + 255) / 256)), dim3(256), 0, s,
                       slots, counts, n_ent, capseg, scan_ws, out, cap);
    return hipGetLastError();
}

// ---- history roll: dst[i] = concat(old[0:hist_rows], fresh[0:fresh_rows])[fresh_rows + i] ----
__global__ void k_hist_roll(uint8_t* dst, const uint8_t* old_hist, const uint8_t* fresh,
                            int64_t hist_rows, int64_t fresh_rows, int64_t row_bytes) {
    const int64_t total = hist_rows * row_bytes;
    for (int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b < total;
         b += (int64_t)gridDim.x * blockDim.x) {
        const int64_t row = b / row_bytes, col = b % row_bytes;
        const int64_t src = fresh_rows + row;  // index into concat
        dst[b] = src < hist_rows ? old_hist[src * row_bytes + col]
                                 : fresh[(src - hist_rows) * row_bytes + col];
    }
}

hipError_t launch_hist_roll(void* dst, const void* old_hist, const void* fresh, int64_t hist_rows,
                            int64_t fresh_rows, int64_t row_bytes, hipStream_t s) {
    const int64_t total = hist_rows * row_bytes;
    const int blocks = (int)((total + 255) / 256 < 1024 ? (total + 255) / 256 : 1024);
    hipLaunchKernelGGL(k_hist_roll, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, s, (uint8_t*)dst,
                       (const uint8_t*)old_hist, (const uint8_t*)fresh, hist_rows, fresh_rows,
                       row_bytes);
    return hipGetLastError();
}

}  // namespace mkid
