// Synthetic ADC stream for tests and the benchmark (NOT part of the hot path).
// out[n] = base[(n0+n) mod 2^16] + AWGN + sum over active pulses of
//          amp_c e^{i theta_c(t)} (e^{i delta(t - start)} - 1)
// base = conj(DAC tone comb) (the loop-back spectrum inversion of ROACH_Setup.py:485-487),
// theta_c(t) = 2 pi (m_c t mod 2^16)/2^16 + phase0_c, delta(tau) = -A (1-e^{-tau/tr}) e^{-tau/tf}
// (pulse shape after ReadoutControls/lib/pulses.py:470-472). Result truncated toward zero (int()).
#include "mkid_internal.h"

namespace mkid {

constexpr int kSynThreads = 256;
constexpr int kSynPerThread = 16;
constexpr int kSynTile = kSynThreads * kSynPerThread;

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

__global__ __launch_bounds__(kSynThreads) void k_synth(int16_t* out, int64_t n, int64_t n0,
                                                       const int16_t* base,
                                                       const mkid_synth_tone* tones,
                                                       const mkid_pulse* pulses, int64_t npulses,
                                                       float tr, float tf, int32_t window,
                                                       float sigma, uint32_t seed) {
    __shared__ int64_t range[2];
    const int64_t t0 = n0 + (int64_t)blockIdx.x * kSynTile;
    if (threadIdx.x == 0) {
        // pulses sorted by start: first with start > t0 - window, first with start >= t0 + tile
        int64_t lo = 0, hi = npulses;
        while (lo < hi) { int64_t m = (lo + hi) / 2; if (pulses[m].start > t0 - window) hi = m; else lo = m + 1; }
        range[0] = lo;
        int64_t lo2 = lo, hi2 = npulses;
        while (lo2 < hi2) { int64_t m = (lo2 + hi2) / 2; if (pulses[m].start >= t0 + kSynTile) hi2 = m; else lo2 = m + 1; }
        range[1] = lo2;
    }
    __syncthreads();
    const int64_t pb = range[0], pe = range[1];
    for (int r = 0; r < kSynPerThread; ++r) {
        const int64_t i = (int64_t)blockIdx.x * kSynTile + r * kSynThreads + threadIdx.x;
        if (i >= n) break;
        const int64_t t = n0 + i;
        float vi = base[2 * (t & 0xffff)], vq = base[2 * (t & 0xffff) + 1];
        if (sigma > 0.f) {
            const uint32_t h1 = hash32((uint32_t)t * 2u + seed * 0x9E3779B9u ^ (uint32_t)(t >> 32));
            const uint32_t h2 = hash32(h1 ^ 0x85ebca6bU);
            const float u1 = ((h1 >> 8) + 1) * (1.0f / 16777217.0f);
            const float u2 = (h2 >> 8) * (1.0f / 16777216.0f);
            const float rad = sigma * sqrtf(-2.f * __logf(u1));
            float sn, cs;
            __sincosf(6.28318530717958647692f * u2, &sn, &cs);
            vi += rad * cs;
            vq += rad * sn;
        }
        for (int64_t p = pb; p < pe; ++p) {
            const mkid_pulse pu = pulses[p];
            const int64_t tau = t - pu.start;
            if (tau < 0 || tau >= window) continue;
            const mkid_synth_tone tn = tones[pu.tone];
            const float ft = (float)tau;
            const float d = -pu.amp_rad * (1.f - __expf(-ft / tr)) * __expf(-ft / tf);
            const uint32_t ph = (uint32_t)((uint64_t)(uint32_t)tn.freq_index * (uint64_t)(t & 0xffff)) & 0xffffu;
            const float th = 6.28318530717958647692f * (float)ph * (1.0f / 65536.0f) + tn.phase0;
            float st, ct, sd, cd;
            sincosf(th, &st, &ct);
            sincosf(d, &sd, &cd);
            // amp e^{i th} (e^{i d} - 1)
            const float er = cd - 1.f, ei = sd;
            vi += tn.amp * (ct * er - st * ei);
            vq += tn.amp * (ct * ei + st * er);
        }
        int qi = (int)vi, qq = (int)vq;  // truncation toward zero, as int() in freqCombLUT
        qi = qi < -32768 ? -32768 : (qi > 32767 ? 32767 : qi);
        qq = qq < -32768 ? -32768 : (qq > 32767 ? 32767 : qq);
        out[2 * i] = (int16_t)qi;
        out[2 * i + 1] = (int16_t)qq;
    }
}

hipError_t launch_synth(int16_t* out, int64_t n, int64_t n0, const int16_t* base,
                        const mkid_synth_tone* tones, const mkid_pulse* pulses, int64_t npulses,
                        float tr, float tf, int32_t window, float sigma, uint32_t seed,
                        hipStream_t s) {
    const int64_t blocks = (n + kSynTile - 1) / kSynTile;
    if (blocks <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_synth, dim3((unsigned)blocks), dim3(kSynThreads), 0, s, out, n, n0, base,
                       tones, pulses, npulses, tr, tf, window, sigma, seed);
    return hipGetLastError();
}

}  // namespace mkid
