// Per-packet optimal-filter pulse height (BASELINE config 5: "per-channel optimal-filter
// pulse-height estimation (fp32)"). The reference computes the pulse template and noise PSD
// (MakeTemplate, pulses.py:239-427) but stubs the filter (pulses.py:398, PulseAnalysis.coeff
// Float32Col(100)); mkid_optimal_filter fills the stub and this kernel applies a per-channel
// filter of that form to the phase stream at every photon packet:
//     h_p = sum_{i < ncoeff} coeff[ch_p][i] * phase[ts_p - pre + i][ch_p]
// One wave per packet: lane l accumulates taps l, l + 64, ... in fp32, then a fixed-order xor
// butterfly over the wave (deterministic). The phase rows of one packet's window are strided by
// C floats, so each lane's read is its own cache line; the volume is small (ncoeff x 4 B per
// packet). Windows that start before the call's first row read the context's carried history of
// the previous call's last rows (mkid_api.hip pulse_heights), so a streamed run loses heights
// only at the stream start and for windows past the call's last row.
#include "mkid_internal.h"

namespace mkid {

constexpr int kHeightWaves = 4;  // packets (waves) per 256-thread workgroup

// Grid-stride over packets: the count can be a device value (the trigger's written count,
// a.d_n) so that a step launches with no host round trip; waves beyond it exit at once.
__global__ __launch_bounds__(64 * kHeightWaves) void k_pulse_heights(HeightArgs a) {
    const int lane = threadIdx.x & 63;
    const int64_t n = a.d_n ? (*a.d_n < a.n ? *a.d_n : a.n) : a.n;
    const int64_t nw = (int64_t)gridDim.x * kHeightWaves;
    for (int64_t p = (int64_t)blockIdx.x * kHeightWaves + (threadIdx.x >> 6); p < n; p += nw) {
        const uint64_t w = a.events[p];
        const int ch = (int)((w >> MKID_PKT_CH_SHIFT) & 0xFFF);
        const int64_t ts = (int64_t)(w & MKID_PKT_TS_MASK);
        // global phase index of the packet: the 28-bit stamp unwrapped into [j0 - 2^27, j0 + 2^27)
        // (a packet emitted at a call's first sample is stamped at the previous call's last row)
        const int64_t base = a.j0 > ((int64_t)1 << 27) ? a.j0 - ((int64_t)1 << 27) : 0;
        const int64_t jg = base + ((ts - (base & (int64_t)MKID_PKT_TS_MASK)) & (int64_t)MKID_PKT_TS_MASK);
        const int64_t r0 = jg - a.j0 - a.pre;  // first phase row of the window (< 0: history)
        const bool inside = ch < a.C && r0 >= -a.hrows && r0 + a.ncoeff <= a.rows;
        float acc = 0.f;
        if (inside) {
            const float* cf = a.coeff + (size_t)ch * a.ncoeff;
            for (int i = lane; i < a.ncoeff; i += 64) {
                const int64_t r = r0 + i;
                const float v = r >= 0 ? a.phase[r * a.C + ch] : a.hist[(a.hrows + r) * a.C + ch];
                acc = fmaf(cf[i], v, acc);
            }
        }
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) acc += __shfl_xor(acc, m, 64);
        if (lane == 0) a.heights[p] = inside ? acc : __builtin_nanf("");
    }
}

hipError_t launch_pulse_heights(const HeightArgs& a, hipStream_t s) {
    if (a.n <= 0) return hipSuccess;
    int64_t blocks = (a.n + kHeightWaves - 1) / kHeightWaves;
    const int64_t cap = (int64_t)(a.ncu > 0 ? a.ncu : 256) * 32;  // 8 waves per SIMD on every CU, then grid-stride
    if (blocks > cap) blocks = cap;
    hipLaunchKernelGGL(k_pulse_heights, dim3((unsigned)blocks), dim3(64 * kHeightWaves), 0, s, a);
    return hipGetLastError();
}

}  // namespace mkid
