// K7-K8: matched filter + baseline (EMA / SVF) + threshold + parabolic peak + dead time +
// packetiser, and the deterministic channel-major compaction of the per-channel event slots.
// Integer semantics are bit-identical to oracle/trigger.c (the oracle header lists the reference
// anchors: ROACH_Pulses.py:59-111, 211-299; set_alpha.py; set_svf.py; set_base_thresh.py;
// Utils/bin.py:5-16; packet fields ROACH_Pulses.py:796-859).
#include "mkid_internal.h"

namespace mkid {

constexpr int kTrigThreads = 64;

__device__ __forceinline__ int32_t clamp16(int32_t v) { return v < -32768 ? -32768 : (v > 32767 ? 32767 : v); }
__device__ __forceinline__ int32_t clampi(int32_t v, int32_t lo, int32_t hi) { return v < lo ? lo : (v > hi ? hi : v); }

__device__ __forceinline__ int64_t peakfit_i(int64_t y1, int64_t y2, int64_t y3) {
    const int64_t den = y3 + y1 - 2 * y2;
    if (den == 0) return y2;
    const int64_t d = y3 - y1;
    return y2 - (d * d) / (8 * den);
}

__device__ __forceinline__ uint64_t pack_wide(int32_t ch, int64_t peak, int32_t base, int64_t j) {
    const uint64_t pk = (uint64_t)clampi((int32_t)((peak >> 4) + 2048), 0, 4095);
    const uint64_t bs = (uint64_t)clampi((base >> 4) + 2048, 0, 4095);
    return ((uint64_t)(ch & 0xFFF) << MKID_PKT_CH_SHIFT) | (pk << MKID_PKT_PEAK_SHIFT) |
           (bs << MKID_PKT_BASE_SHIFT) | ((uint64_t)j & MKID_PKT_TS_MASK);
}

enum { ST_ARMED = 0, ST_PULSE = 1, ST_DEAD = 2, ST_REARM = 3 };

// One thread per channel, sequential in time (v1). The 26-sample matched-filter window is a
// register ring indexed statically inside 26-sample unrolled groups.
__global__ __launch_bounds__(kTrigThreads) void k_trigger(TrigArgs a) {
    const int c = blockIdx.x * kTrigThreads + threadIdx.x;
    if (c >= a.C) return;
    const int C = a.C;
    int32_t tap[kFirTaps];
#pragma unroll
    for (int i = 0; i < kFirTaps; ++i) tap[i] = a.fir[c * kFirTaps + i];
    const int32_t thr = a.thr[c];
    TrigState s = a.st[c];
    int32_t win[kFirTaps];
    win[0] = 0;
#pragma unroll
    for (int i = 1; i < kFirTaps; ++i) win[i] = a.rhist[(i - 1) * C + c];  // raw_{i-26}
    int32_t n = 0;
    uint64_t* slot = a.slots + (int64_t)c * a.capc;

    for (int64_t g = 0; g < a.J; g += kFirTaps) {
        const int64_t left = a.J - g;
#pragma unroll
        for (int u = 0; u < kFirTaps; ++u) {
            if (u >= left) continue;  // tail group only; keeps the loop fully unrolled
            const int64_t j = g + u;
            win[u] = a.raw[j * C + c];
            int32_t acc = 0;
#pragma unroll
            for (int i = 0; i < kFirTaps; ++i) acc += tap[i] * win[(u - i + kFirTaps) % kFirTaps];
            const int32_t f = clamp16(acc >> 11);
            if (!s.binit) {
                s.B = (a.mode == MKID_BASE_NONE) ? 0 : f;
                s.low = (int64_t)f << 16;
                s.band = 0;
                s.binit = 1;
            }
            const int32_t base_prev = (a.mode == MKID_BASE_SVF) ? (int32_t)(s.low >> 16) : s.B;
            const int32_t e = f - base_prev;
            const bool gate = (a.base_thr <= 0) || (e < a.base_thr && e > -a.base_thr);
            if (a.mode == MKID_BASE_EMA && gate) {
                s.B += (a.alpha * e) >> 9;
            } else if (a.mode == MKID_BASE_SVF && gate) {
                const int64_t high = ((int64_t)f << 16) - s.low - (((int64_t)a.kq * s.band) >> 16);
                s.band += ((int64_t)a.kf * high) >> 16;
                s.low += ((int64_t)a.kf * s.band) >> 16;
            }
            if (s.st == ST_ARMED) {
                if (e < thr) s.st = ST_PULSE;
            } else if (s.st == ST_PULSE) {
                if (f > s.f1) {
                    const int64_t pk = peakfit_i(s.f2, s.f1, f);
                    if (n < a.capc) slot[n] = pack_wide(c, pk, base_prev, a.j0 + j - 1);
                    ++n;
                    s.st = ST_DEAD;
                    s.cnt = a.dead;
                }
            } else if (s.st == ST_DEAD) {
                s.cnt -= 1;
                if (s.cnt <= 0) s.st = ST_REARM;
            } else {
                if (e >= thr) s.st = ST_ARMED;
            }
            s.f2 = s.f1;
            s.f1 = f;
        }
    }
    a.st[c] = s;
    a.counts[c] = n;
}

hipError_t launch_trigger(const TrigArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_trigger, dim3((a.C + kTrigThreads - 1) / kTrigThreads), dim3(kTrigThreads),
                       0, s, a);
    return hipGetLastError();
}

// ---- compaction: exclusive scan of per-channel counts (one block), then per-channel copy ----
constexpr int kScanThreads = 1024;

// d_counts[0] accumulates packets produced, d_counts[1] packets stored in `out` (<= cap), over
// the sub-chunks of one process call (zeroed by the caller at the start of the call).
__global__ __launch_bounds__(kScanThreads) void k_scan_counts(const int32_t* counts, int32_t C,
                                                              int32_t capc, int64_t cap,
                                                              int64_t* offs, int64_t* d_counts) {
    __shared__ int64_t part[kScanThreads];
    __shared__ unsigned long long tot;
    const int64_t prev = d_counts[1];
    const int per = (C + kScanThreads - 1) / kScanThreads;
    const int b = threadIdx.x * per;
    int64_t sum = 0, sumw = 0;
    for (int i = 0; i < per; ++i)
        if (b + i < C) { const int v = counts[b + i]; sum += v; sumw += v < capc ? v : capc; }
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
    for (int i = 0; i < per; ++i)
        if (b + i < C) { offs[b + i] = run; const int v = counts[b + i]; run += v < capc ? v : capc; }
    atomicAdd(&tot, (unsigned long long)sum);
    __syncthreads();
    if (threadIdx.x == 0) {
        d_counts[0] += (int64_t)tot;
        const int64_t w = prev + part[kScanThreads - 1];
        d_counts[1] = w < cap ? w : cap;
    }
}

__global__ __launch_bounds__(256) void k_gather_events(const uint64_t* slots, const int32_t* counts,
                                                       int32_t capc, const int64_t* offs,
                                                       uint64_t* out, int64_t cap) {
    const int c = blockIdx.x;
    const int n = counts[c] < capc ? counts[c] : capc;
    const int64_t o = offs[c];
    for (int i = threadIdx.x; i < n; i += blockDim.x)
        if (o + i < cap) out[o + i] = slots[(int64_t)c * capc + i];
}

hipError_t launch_compact(const uint64_t* slots, const int32_t* counts, int32_t C, int32_t capc,
                          uint64_t* out, int64_t cap, int64_t* d_counts, int64_t* scan_ws,
                          hipStream_t s) {
    hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(kScanThreads), 0, s, counts, C, capc, cap,
                       scan_ws, d_counts);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_gather_events, dim3(C), dim3(256), 0, s, slots, counts, capc, scan_ws,
                       out, cap);
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
