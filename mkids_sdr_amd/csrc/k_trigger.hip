// K7-K8: matched filter + baseline (EMA / SVF) + threshold + parabolic peak + dead time +
// packetiser, evaluated EXACTLY but in parallel over time by speculative segments:
//
//   k_trig_spec  thread = (channel c, segment s of L phase samples). Segment 0 starts from the
//                channel's carried state (exact). Segment s>0 starts W samples early from a guessed
//                state (re-arm pending, baseline = first filtered sample), runs the warm-up
//                silently, records its state S_spec at the segment start, then emits packets.
//   k_trig_fix   thread = channel. Walks the segments in order with the true state T. If
//                T == S_spec (canonical compare) the segment's packets are exact. Otherwise it
//                re-runs the true and the speculative trajectories side by side from the segment
//                start until they coincide (the recurrence is deterministic in (state, input)), and
//                splices: true packets before the merge + speculative packets after it.
//   compaction   exclusive scan over (channel, segment) counts -> channel-major, time-ascending.
//
// The result is bit-identical to the sequential oracle/trigger.c for every input; the speculation
// only decides how much sequential work the fix-up does (EMA merges within ~10^2 samples on noisy
// phase). SVF mode (slow 2-pole baseline with a wide dead band) uses one segment = serial.
#include "trig_common.h"

namespace mkid {

constexpr int kTrigThreads = 64;

struct Win {
    int32_t w[kFirTaps];
};

// Prologue: load raw_{j-25..j-1} into ring slots (j' - j + 26) % 26 for a ring aligned at j.
__device__ __forceinline__ void load_window(Win& win, const TrigSpecArgs& a, int c, int64_t j) {
    win.w[0] = 0;
#pragma unroll
    for (int i = 1; i < kFirTaps; ++i) {
        const int64_t jj = j - kFirTaps + i;  // slot i holds raw_{j-26+i}
        win.w[i] = jj >= 0 ? a.raw[jj * a.C + c] : (jj >= -kRawHist ? a.rhist[(jj + kRawHist) * a.C + c] : 0);
    }
}

__global__ __launch_bounds__(kTrigThreads) void k_trig_spec(TrigSpecArgs a) {
    const int c = blockIdx.x * kTrigThreads + threadIdx.x;
    const int s = blockIdx.y;
    if (c >= a.C) return;
    const int C = a.C;
    int32_t tap[kFirTaps];
#pragma unroll
    for (int i = 0; i < kFirTaps; ++i) tap[i] = a.fir[c * kFirTaps + i];
    const TrigCfg k{a.thr[c], a.mode, a.alpha, a.kf, a.kq, a.base_thr, a.dead};
    const int64_t seg0 = (int64_t)s * a.L;
    const int64_t seg1 = seg0 + a.L < a.J ? seg0 + a.L : a.J;
    const int64_t jw = s == 0 ? 0 : seg0 - a.W;
    TrigState st;
    if (s == 0) {
        st = a.st_in[c];
    } else {
        st = TrigState{0, 0, ST_REARM, 0, 0, 0, 0, 0, 0, 0};
    }
    Win win;
    load_window(win, a, c, jw);
    const int64_t sc = (int64_t)c * a.nseg + s;
    uint64_t* slot = a.slots + sc * a.capseg;
    int32_t n = 0;
    for (int64_t g = jw; g < seg1; g += kFirTaps) {
        const int64_t left = seg1 - g;
#pragma unroll
        for (int u = 0; u < kFirTaps; ++u) {
            if (u >= left) continue;
            const int64_t j = g + u;
            win.w[u] = a.raw[j * C + c];
            int32_t acc = 0;
#pragma unroll
            for (int i = 0; i < kFirTaps; ++i) acc += tap[i] * win.w[(u - i + kFirTaps) % kFirTaps];
            if (s > 0 && j == seg0) a.s_spec[(int64_t)s * C + c] = st;
            uint64_t pkt;
            if (trig_step(st, mf_out(acc), k, c, a.j0 + j, &pkt) && j >= seg0) {
                if (n < a.capseg) slot[n] = pkt;
                ++n;
            }
        }
    }
    a.s_end[(int64_t)s * C + c] = st;
    a.counts[sc] = n;
}

__global__ __launch_bounds__(kTrigThreads) void k_trig_fix(TrigSpecArgs a) {
    const int c = blockIdx.x * kTrigThreads + threadIdx.x;
    if (c >= a.C) return;
    const int C = a.C;
    int32_t tap[kFirTaps];
#pragma unroll
    for (int i = 0; i < kFirTaps; ++i) tap[i] = a.fir[c * kFirTaps + i];
    const TrigCfg k{a.thr[c], a.mode, a.alpha, a.kf, a.kq, a.base_thr, a.dead};
    TrigState T = a.s_end[c];  // segment 0 is exact
    uint64_t* scratch = a.scratch + (int64_t)c * a.capseg;
    int32_t reruns = 0;
    for (int s = 1; s < a.nseg; ++s) {
        const TrigState S0 = a.s_spec[(int64_t)s * C + c];
        if (state_eq(T, S0, a.mode)) {
            T = a.s_end[(int64_t)s * C + c];
            continue;
        }
        ++reruns;
        const int64_t seg0 = (int64_t)s * a.L;
        const int64_t seg1 = seg0 + a.L < a.J ? seg0 + a.L : a.J;
        TrigState tru = T, spc = S0;
        int32_t nt = 0, ndrop = 0;
        bool merged = false;
        Win win;
        load_window(win, a, c, seg0);
        for (int64_t g = seg0; g < seg1 && !merged; g += kFirTaps) {
            const int64_t left = seg1 - g;
#pragma unroll
            for (int u = 0; u < kFirTaps; ++u) {
                if (u >= left || merged) continue;
                const int64_t j = g + u;
                win.w[u] = a.raw[j * C + c];
                int32_t acc = 0;
#pragma unroll
                for (int i = 0; i < kFirTaps; ++i) acc += tap[i] * win.w[(u - i + kFirTaps) % kFirTaps];
                const int32_t f = mf_out(acc);
                uint64_t pkt;
                if (trig_step(tru, f, k, c, a.j0 + j, &pkt)) {
                    if (nt < a.capseg) scratch[nt] = pkt;
                    ++nt;
                }
                uint64_t dummy;
                if (trig_step(spc, f, k, c, a.j0 + j, &dummy)) ++ndrop;
                merged = state_eq(tru, spc, a.mode);
            }
        }
        const int64_t sc = (int64_t)c * a.nseg + s;
        uint64_t* slot = a.slots + sc * a.capseg;
        const int32_t cnt = a.counts[sc] < a.capseg ? a.counts[sc] : a.capseg;
        int32_t total = nt;
        if (merged) {
            const int32_t keep = cnt - ndrop;  // speculative packets after the merge point
            if (nt < ndrop) {
                for (int32_t i = 0; i < keep; ++i) slot[nt + i] = slot[ndrop + i];
            } else if (nt > ndrop) {
                for (int32_t i = keep - 1; i >= 0; --i)
                    if (nt + i < a.capseg) slot[nt + i] = slot[ndrop + i];
            }
            total = nt + (a.counts[sc] - ndrop);
            T = a.s_end[(int64_t)s * C + c];
        } else {
            T = tru;
        }
        for (int32_t i = 0; i < nt && i < a.capseg; ++i) slot[i] = scratch[i];
        a.counts[sc] = total;
    }
    a.st_out[c] = T;
    if (a.reruns) a.reruns[c] = reruns;
}

hipError_t launch_trigger(const TrigSpecArgs& a, hipStream_t s) {
    const unsigned cb = (a.C + kTrigThreads - 1) / kTrigThreads;
    hipLaunchKernelGGL(k_trig_spec, dim3(cb, a.nseg), dim3(kTrigThreads), 0, s, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_trig_fix, dim3(cb), dim3(kTrigThreads), 0, s, a);
    return hipGetLastError();
}

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
