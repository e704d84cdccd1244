// K5-K6: per-channel 26-tap IQ low-pass with decimation by 2, IQ-centre subtraction, atan2,
// Fix16_13 quantisation.
//   y_j = sum_i g_i z_{2j+1-i}                  (taps int(lpf*(2**11-1))/2^11, ROACH_Pulses.py:69,88)
//   phi_j = atan2(Im y - qc, Re y - ic)          (pulse_triggering_IQ.py:152, conv_phase_centers)
//   computed centred: y - c = sum_i g_i (z_i - c') + r  (mkid_internal.h Centring)
//   raw_j = clamp(rint(phi_j * 2^13), +-25736)   (Fix16_13, ROACH_Pulses.py:274-278)
// Thread = one channel x JB = 13*kLpfRounds consecutive outputs: a 26-deep register window slides
// by 2 frames per output; slots are static inside each 13-output round, so z is read from HBM
// once plus a 25-frame prologue per thread (25/(2 JB) re-read). Lanes = consecutive channels:
// every z load / phase store of a wave is one contiguous 512 B / 256 B segment.
#include "fft_common.h"
#include "mkid_internal.h"

namespace mkid {

constexpr int kLpfThreads = 256;
constexpr int kLpfRounds = 8;
constexpr int kLpfJB = 13 * kLpfRounds;  // outputs per thread

__global__ __launch_bounds__(kLpfThreads) void k_lpf_phase(LpfArgs a) {
    const int c = blockIdx.y * kLpfThreads + threadIdx.x;
    if (c >= a.C) return;
    const int64_t j0 = (int64_t)blockIdx.x * kLpfJB;
    const int C = a.C;
    const float2 ncen = a.cen.ncen[c], cor = a.cen.cor[c];   // centred low-pass (mkid_internal.h)

    // slot s holds frame f with (f - fbase) % 26 == s ; fbase = 2*j0 + 1 - 25
    float2 w[kFirTaps];
    const int64_t fbase = 2 * j0 + 1 - (kFirTaps - 1);
#pragma unroll
    for (int i = 0; i < kFirTaps - 1; ++i) {
        const int64_t f = fbase + i;
        const float2 v = f >= 0 ? a.z[f * C + c] : a.zhist[(f + kLpfHist) * C + c];
        w[i] = make_float2(v.x + ncen.x, v.y + ncen.y);
    }
    float2 ys = make_float2(0.f, 0.f);
    for (int rd = 0; rd < kLpfRounds; ++rd) {
        const int64_t jr = j0 + 13 * rd;
        if (jr >= a.J) break;
#pragma unroll
        for (int u = 0; u < 13; ++u) {
            const int64_t j = jr + u;
            if (j < a.J) {
                const int64_t f1 = 2 * j + 1;
                const int s1 = (2 * u + kFirTaps - 1) % kFirTaps;  // slot of frame 2j+1
                const int s0 = (2 * u + kFirTaps - 2) % kFirTaps;  // slot of frame 2j
                if (u > 0 || rd > 0) {
                    const float2 v0 = a.z[(f1 - 1) * C + c];
                    w[s0] = make_float2(v0.x + ncen.x, v0.y + ncen.y);
                }
                const float2 v1 = a.z[f1 * C + c];
                w[s1] = make_float2(v1.x + ncen.x, v1.y + ncen.y);
                float yr = 0.f, yi = 0.f;
#pragma unroll
                for (int i = 0; i < kFirTaps; ++i) {
                    const int s = (2 * u + kFirTaps - 1 - i + kFirTaps) % kFirTaps;  // frame 2j+1-i
                    yr = fmaf(a.taps.g[i], w[s].x, yr);
                    yi = fmaf(a.taps.g[i], w[s].y, yi);
                }
                ys.x += yr;
                ys.y += yi;
                const float ph = phase_atan2(yi + cor.y, yr + cor.x);
                int q = __float2int_rn(ph * 8192.0f);
                q = q < -25736 ? -25736 : (q > 25736 ? 25736 : q);
                if (a.phase) a.phase[j * C + c] = ph;
                a.raw[j * C + c] = (int16_t)q;
                if (c == a.iq_ch && a.iqtap) {
                    a.iqtap[2 * j] = iq16(yr + a.cen.tap_off.x);
                    a.iqtap[2 * j + 1] = iq16(yi + a.cen.tap_off.y);
                }
            }
        }
    }
    if (a.ysum) {
        ysum_add(a.ysum, c, ys.x, ys.y);
    }
}

hipError_t launch_lpf_phase(const LpfArgs& a, hipStream_t s) {
    if (a.J <= 0) return hipSuccess;
    dim3 grid((unsigned)((a.J + kLpfJB - 1) / kLpfJB), (a.C + kLpfThreads - 1) / kLpfThreads);
    hipLaunchKernelGGL(k_lpf_phase, grid, dim3(kLpfThreads), 0, s, a);
    return hipGetLastError();
}

}  // namespace mkid
