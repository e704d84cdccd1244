// K1-K4: polyphase filter bank + N-point FFT (2x oversampled, hop M = N/2) + bin select + DDC.
//
// One 256-thread workgroup owns FPB = 256/NT frame slots (NT = N/PTS threads per frame, PTS
// points per thread) and walks FL consecutive frame groups. Per frame:
//   PFB   u[p] = sum_tau h[tau N + p] x[(k+1)M - TN + tau N + p]     (p = t + r NT: coalesced)
//   FFT   Stockham radix-16/8/4 passes, butterflies in registers, exchanges through padded LDS
//   K3/4  z[k][c] = X[bin_c] * (-1)^(bin_c (k+1)) * conj(LUT_c[k mod P]) / 2^15
// Reference geometry: fft_len/channels ROACH_Setup.py:507,515; bins ROACH_Setup.py:534-550; DDS
// LUT at 2 fs/N ROACH_Setup.py:525. Taps/window of the PFB: build decision (firmware absent).
#include "fft_common.h"
#include "mkid_internal.h"

namespace mkid {

constexpr int kChanThreads = 256;
constexpr int kFramesPerIter = 8;  // FL

template <int N>
__global__ __launch_bounds__(kChanThreads) void k_channelize(ChanArgs a) {
    using PL = Plan<N>;
    constexpr int PTS = PL::PTS, NT = N / PTS, FPB = kChanThreads / NT;
    constexpr int M = N / 2, C = N / 2, T = kPfbTaps, H = T * N - M;
    constexpr int LDSF = lds_frame_elems<N>();
    constexpr int CPT = C / NT;  // channels per thread in the select stage
    __shared__ float2 lds[FPB * LDSF];

    const int slot = threadIdx.x / NT;
    const int t = threadIdx.x % NT;
    float2* buf = lds + slot * LDSF;

    Twiddle<N, PTS, PL::R2, PL::R1> tw2;
    tw2.init(t);
    Twiddle<N, PTS, (PL::NP == 3 ? PL::R3 : 2), PL::R1 * PL::R2> tw3;
    if constexpr (PL::NP == 3) tw3.init(t);

    int32_t bin[CPT];
#pragma unroll
    for (int q = 0; q < CPT; ++q) bin[q] = a.bins[t + q * NT];

    const int64_t kbase = (int64_t)blockIdx.x * FPB * kFramesPerIter;
    for (int it = 0; it < kFramesPerIter; ++it) {
        const int64_t k = kbase + (int64_t)it * FPB + slot;
        const bool valid = k < a.K;
        const int64_t kk = valid ? k : a.K - 1;

        // ---- PFB ----
        float2 v[PTS];
        const int64_t n0 = (kk + 1) * M - (int64_t)T * N;
#pragma unroll
        for (int r = 0; r < PTS; ++r) {
            const int p = t + r * NT;
            float ur = 0.f, ui = 0.f;
#pragma unroll
            for (int tau = 0; tau < T; ++tau) {
                const int64_t n = n0 + tau * N + p;
                const uint32_t w = n >= 0 ? a.x[n] : a.xhist[n + H];
                const float h = a.pfb[tau * N + p];
                ur = fmaf(h, (float)(int16_t)(w & 0xffffu), ur);
                ui = fmaf(h, (float)(int16_t)(w >> 16), ui);
            }
            v[r] = make_float2(ur, ui);
        }

        // ---- FFT ----
        st_dft<PTS, PL::R1>(v);
        st_write<N, PTS, PL::R1, 1>(buf, v, t);
        __syncthreads();
        st_read<N, PTS, PL::R2>(buf, v, t);
        __syncthreads();
        tw2.apply(v);
        st_dft<PTS, PL::R2>(v);
        st_write<N, PTS, PL::R2, PL::R1>(buf, v, t);
        __syncthreads();
        if constexpr (PL::NP == 3) {
            st_read<N, PTS, PL::R3>(buf, v, t);
            __syncthreads();
            tw3.apply(v);
            st_dft<PTS, PL::R3>(v);
            st_write<N, PTS, PL::R3, PL::R1 * PL::R2>(buf, v, t);
            __syncthreads();
        }

        // ---- bin select + DDC ----
        const int64_t kg = a.k0 + kk;
        const int podd = (int)((kg + 1) & 1);
        const int lidx = (int)(kg & (a.P - 1));
#pragma unroll
        for (int q = 0; q < CPT; ++q) {
            const int c = t + q * NT;
            float2 X = buf[lpad(bin[q])];
            if (podd & bin[q] & 1) X = make_float2(-X.x, -X.y);
            const float2 lo = a.lo[(int64_t)c * a.P + lidx];
            if (valid) a.z[kk * C + c] = cmul(X, lo);
        }
        __syncthreads();
    }
}

bool channelize_supported(int N) {
    return N == 128 || N == 256 || N == 512 || N == 1024 || N == 2048 || N == 4096;
}

template <int N>
static hipError_t launch_n(const ChanArgs& a, hipStream_t s) {
    constexpr int NT = N / Plan<N>::PTS, FPB = kChanThreads / NT;
    const int64_t per_block = (int64_t)FPB * kFramesPerIter;
    const int64_t blocks = (a.K + per_block - 1) / per_block;
    if (blocks <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_channelize<N>, dim3((unsigned)blocks), dim3(kChanThreads), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_channelize(int N, const ChanArgs& a, hipStream_t s) {
    switch (N) {
        case 128: return launch_n<128>(a, s);
        case 256: return launch_n<256>(a, s);
        case 512: return launch_n<512>(a, s);
        case 1024: return launch_n<1024>(a, s);
        case 2048: return launch_n<2048>(a, s);
        case 4096: return launch_n<4096>(a, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace mkid
