// K1-K4: polyphase filter bank + N-point FFT (2x oversampled, hop M = N/2) + bin select + DDC.
//
// A workgroup of BT threads owns a contiguous run of frames and walks it FPB frames at a time
// (NT = N/PTS threads per frame, PTS = 8 points per thread, FPB = BT/NT):
//   input  ring of RS = 2T-1+FPB hops of M int16 I/Q samples in LDS. Each iteration brings FPB
//          new hops with ONE 16-byte global load per thread, issued one iteration ahead so its
//          latency hides behind the FFT; each sample is read from HBM once (+ (2T-1)/run warm-up).
//   PFB    u[p] = sum_tau h[tau N + p] x[(k+1)M - TN + tau N + p]  (h in registers, x from LDS)
//   FFT    Stockham radix-8/4 passes, butterflies in registers, one twiddle base per butterfly
//          (powers rebuilt in registers), exchanges through padded LDS. With MKID_CHAN_DBUF the
//          passes ping-pong between two LDS buffers: one barrier per pass instead of two.
//   K3/4   z[k][c] = X[bin_c] (-1)^(bin_c (k+1)) conj(LUT_c[k mod P]) / 2^15; LO table [P][C] so
//          both the LO row and the z row of a frame are contiguous (coalesced)
// Reference geometry: fft_len/channels ROACH_Setup.py:507,515; bins ROACH_Setup.py:534-550; DDS
// LUT at 2 fs/N ROACH_Setup.py:525. Taps/window of the PFB: build decision (firmware absent).
#include "fft_common.h"
#include "mkid_internal.h"

#ifndef MKID_CHAN_MINWAVES
#define MKID_CHAN_MINWAVES 1
#endif
#ifndef MKID_CHAN_DBUF
#define MKID_CHAN_DBUF 1
#endif

namespace mkid {

constexpr int kPts = 8;

template <int N>
struct Geo {
    static constexpr int PTS = kPts, NT = N / PTS;
    static constexpr int BT = NT > 256 ? NT : 256;     // threads per workgroup
    static constexpr int FPB = BT / NT;                 // frames in flight per workgroup
    static constexpr int M = N / 2, C = N / 2, T = kPfbTaps;
    static constexpr int RS = 2 * T - 1 + FPB;          // ring slots (hops)
    static constexpr int LDSF = lds_frame_elems<N>();
    static constexpr int NBUF = MKID_CHAN_DBUF ? 2 : 1;  // FFT exchange buffers per frame
    static constexpr int CPT = C / NT;                  // channels per thread in select
    static constexpr int NEW = FPB * M;                 // new samples per iteration
    static constexpr int SPT = NEW / BT;                // new samples per thread (4)
    static_assert(SPT == 4, "one 16-byte load per thread per iteration");
    static constexpr int NS2 = Plan8<N>::R[0], NS3 = NS2 * Plan8<N>::R[1], NS4 = NS3 * Plan8<N>::R[2];
    static constexpr size_t lds_bytes = (size_t)RS * M * 4 + (size_t)FPB * NBUF * LDSF * 8;
};

// Load the 16 bytes (4 samples) this thread contributes to the FPB hops starting at first_hop.
template <int N>
__device__ __forceinline__ uint4 load_new(const ChanArgs& a, int64_t first_hop, int tid) {
    using G = Geo<N>;
    const int64_t s0 = first_hop * G::M + (int64_t)tid * G::SPT;  // sample index in chunk
    if (s0 >= (int64_t)a.K * G::M) return make_uint4(0, 0, 0, 0);
    if (s0 >= -a.avail) return *reinterpret_cast<const uint4*>(a.x + s0);
    const int64_t hs = s0 + a.avail + (G::T * N - G::M);  // into xhist (H = TN - M samples)
    return *reinterpret_cast<const uint4*>(a.xhist + hs);
}

template <int N>
__global__ __launch_bounds__(Geo<N>::BT, MKID_CHAN_MINWAVES) void k_channelize(ChanArgs a) {
    using G = Geo<N>;
    using PL = Plan8<N>;
    constexpr int PTS = G::PTS, NT = G::NT, M = G::M, C = G::C, T = G::T, RS = G::RS;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t* ring = reinterpret_cast<uint32_t*>(smem);
    float2* fbuf = reinterpret_cast<float2*>(smem + (size_t)RS * M * 4);

    const int tid = threadIdx.x;
    const int slot = tid / NT;
    const int t = tid % NT;
    float2* bufA = fbuf + slot * G::NBUF * G::LDSF;
    [[maybe_unused]] float2* bufB = bufA + (G::NBUF - 1) * G::LDSF;  // == bufA without double buffering

    // PFB taps for this thread's points (constant over frames)
    float h[T][PTS];
#pragma unroll
    for (int tau = 0; tau < T; ++tau)
#pragma unroll
        for (int r = 0; r < PTS; ++r) h[tau][r] = a.pfb[tau * N + t + r * NT];

    TwiddleRec<N, PTS, PL::R[1], G::NS2> tw2;
    tw2.init(t);
    TwiddleRec<N, PTS, PL::R[2], G::NS3> tw3;
    tw3.init(t);
    TwiddleRec<N, PTS, (PL::NP == 4 ? PL::R[3] : 2), G::NS4> tw4;
    if constexpr (PL::NP == 4) tw4.init(t);

    int32_t bin[G::CPT];
#pragma unroll
    for (int q = 0; q < G::CPT; ++q) bin[q] = a.bins[t + q * NT];

    const int64_t k_begin = (int64_t)blockIdx.x * a.frames_per_block;
    int64_t k_end = k_begin + a.frames_per_block;
    if (k_end > a.K) k_end = a.K;
    if (k_begin >= k_end) return;

    // prologue: hops k_begin-2T+1 .. k_begin+FPB-1 -> ring (slot = hop mod RS)
    {
        const int64_t h0 = k_begin - 2 * T + 1;
        for (int g = 0; g < RS; g += G::FPB) {
            const int64_t hop = h0 + g + (tid * G::SPT) / M;
            if (hop > h0 + RS - 1) continue;  // RS need not be a multiple of FPB
            const uint4 v = load_new<N>(a, h0 + g, tid);
            const int off = (tid * G::SPT) % M;
            *reinterpret_cast<uint4*>(ring + (int)(((hop % RS) + RS) % RS) * M + off) = v;
        }
    }
    uint4 pre = load_new<N>(a, k_begin + G::FPB, tid);  // next iteration's hops
    __syncthreads();

    for (int64_t kb = k_begin; kb < k_end; kb += G::FPB) {
        const int64_t k = kb + slot;  // this thread's frame
        // ---- PFB from the LDS ring ----
        const int64_t h_first = k + 1 - 2 * T;  // oldest hop of frame k
        const int sb = (int)(((h_first % RS) + RS) % RS);
        float2 v[PTS];
#pragma unroll
        for (int r = 0; r < PTS; ++r) {
            const int p = t + r * NT;
            const int hi = p / M, off = p % M;
            float ur = 0.f, ui = 0.f;
#pragma unroll
            for (int tau = 0; tau < T; ++tau) {
                int sl = sb + 2 * tau + hi;  // < 2 RS
                sl -= sl >= RS ? RS : 0;
                const uint32_t w = ring[sl * M + off];
                ur = fmaf(h[tau][r], (float)(int16_t)(w & 0xffffu), ur);
                ui = fmaf(h[tau][r], (float)(int16_t)(w >> 16), ui);
            }
            v[r] = make_float2(ur, ui);
        }
        st_dft<PTS, PL::R[0]>(v);
#if MKID_CHAN_DBUF
        // pass 1 -> A. The barrier publishes A and retires every ring read of this iteration.
        st_write<N, PTS, PL::R[0], 1>(bufA, v, t);
        __syncthreads();
        {
            const int64_t hop = kb + G::FPB + (tid * G::SPT) / M;
            *reinterpret_cast<uint4*>(ring + (int)(hop % RS) * M + (tid * G::SPT) % M) = pre;
            pre = load_new<N>(a, kb + 2 * G::FPB, tid);
        }
        st_read<N, PTS, PL::R[1]>(bufA, v, t);
        tw2.apply(v);
        st_dft<PTS, PL::R[1]>(v);
        st_write<N, PTS, PL::R[1], G::NS2>(bufB, v, t);
        __syncthreads();
        st_read<N, PTS, PL::R[2]>(bufB, v, t);
        tw3.apply(v);
        st_dft<PTS, PL::R[2]>(v);
        st_write<N, PTS, PL::R[2], G::NS3>(bufA, v, t);
        __syncthreads();
        const float2* fin = bufA;
        if constexpr (PL::NP == 4) {
            st_read<N, PTS, PL::R[3]>(bufA, v, t);
            tw4.apply(v);
            st_dft<PTS, PL::R[3]>(v);
            st_write<N, PTS, PL::R[3], G::NS4>(bufB, v, t);
            __syncthreads();
            fin = bufB;
        }
#else
        __syncthreads();  // all PFB reads of the oldest FPB hops are done
        {
            const int64_t hop = kb + G::FPB + (tid * G::SPT) / M;
            *reinterpret_cast<uint4*>(ring + (int)(hop % RS) * M + (tid * G::SPT) % M) = pre;
            pre = load_new<N>(a, kb + 2 * G::FPB, tid);
        }
        st_write<N, PTS, PL::R[0], 1>(bufA, v, t);
        __syncthreads();
        st_read<N, PTS, PL::R[1]>(bufA, v, t);
        __syncthreads();
        tw2.apply(v);
        st_dft<PTS, PL::R[1]>(v);
        st_write<N, PTS, PL::R[1], G::NS2>(bufA, v, t);
        __syncthreads();
        st_read<N, PTS, PL::R[2]>(bufA, v, t);
        __syncthreads();
        tw3.apply(v);
        st_dft<PTS, PL::R[2]>(v);
        st_write<N, PTS, PL::R[2], G::NS3>(bufA, v, t);
        __syncthreads();
        if constexpr (PL::NP == 4) {
            st_read<N, PTS, PL::R[3]>(bufA, v, t);
            __syncthreads();
            tw4.apply(v);
            st_dft<PTS, PL::R[3]>(v);
            st_write<N, PTS, PL::R[3], G::NS4>(bufA, v, t);
            __syncthreads();
        }
        const float2* fin = bufA;
#endif
        // ---- bin select + DDC ----
        if (k < k_end) {
            const int64_t kg = a.k0 + k;
            const int lidx = (int)(kg & (a.P - 1));
#pragma unroll
            for (int q = 0; q < G::CPT; ++q) {
                const int c = t + q * NT;
                float2 X = fin[lpad(bin[q])];
                const float2 lo = a.lo[lidx * C + c];
                a.z[k * C + c] = cmul(X, lo);
            }
        }
        // Double-buffered: the next iteration's first LDS write goes to A before any barrier.
        // With 4 passes the select above read B (safe); with 3 it read A: barrier first. (Single
        // buffer: the next write follows the post-PFB barrier.)
        if constexpr (MKID_CHAN_DBUF && PL::NP != 4) __syncthreads();
    }
}

bool channelize_supported(int N) {
    return N == 128 || N == 256 || N == 512 || N == 1024 || N == 2048 || N == 4096;
}

template <int N>
static hipError_t launch_n(const ChanArgs& a0, hipStream_t s) {
    using G = Geo<N>;
    static std::atomic<uint64_t> attr_mask{0};
    hipError_t e = ensure_lds_attr(attr_mask, (const void*)k_channelize<N>, (int)G::lds_bytes);
    if (e != hipSuccess) return e;
    ChanArgs a = a0;
    if (a.K <= 0) return hipSuccess;
    // contiguous frame runs: long enough to amortise the (2T-1)-hop warm-up, enough runs to
    // give every CU several workgroups
    int64_t fpb = a.K / 2048;
    fpb = fpb < 64 ? 64 : (fpb > 1024 ? 1024 : fpb);
    fpb = (fpb + G::FPB - 1) / G::FPB * G::FPB;
    a.frames_per_block = fpb;
    const int64_t blocks = (a.K + fpb - 1) / fpb;
    hipLaunchKernelGGL(k_channelize<N>, dim3((unsigned)blocks), dim3(G::BT), G::lds_bytes, s, a);
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
