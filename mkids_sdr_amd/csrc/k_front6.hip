// Fused front end k_front6 (N = 2048, config 3/4): k_front3's wave-specialised arithmetic at ONE
// frame per iteration, in a 768-thread workgroup small enough that TWO of them share a CU.
//
// Why (round 4): k_front3's 16 waves per CU (one workgroup, 120 KB of LDS) run
// latency-bound, not issue-bound: stamps put the four waves of a SIMD at 2.5-3.4 k work cycles per
// 3.9 k-cycle iteration, each waiting 0.7-0.9 k cycles at the one barrier per iteration, and PMC
// at ~0.18 VALU wave-instructions per SIMD cycle (37 % of the SIMD-32 issue rate); removing 8.5 % of
// the VALU instructions (a pair ring) or giving a transform wave two independent sub-FFTs did not
// shorten it. Two independent workgroups per CU give each SIMD 6 waves from two barrier domains:
// while one workgroup's waves wait at their barrier, the other's run.
//
//   workgroup  4 transform waves (sub-FFT w of the iteration's frame k) + 8 select waves (frame
//              k - 1, two channels per thread in k_front3's select-slot order), 768 threads
//   ring       9 hops (frame k reads hops k-7 .. k; the hop k+1 prefetched at the loop top is
//              written over hop k-8), paired planes (ring3_idx) as k_front3: 36 KiB
//   Y          [2][4][576] float2 (iteration t writes buffer t & 1, the select reads (t-1) & 1): 36 KiB
//   tables     stage-1/2 twiddles (read from LDS: registers are 80 per thread at 6 waves per SIMD)
// 75.9 KiB per workgroup, two per CU. The select loop is unrolled into (accumulate, output) frame
// pairs so the low-pass accumulators never meet in a branch's phi nodes (the k_front5 lesson), and
// the NW-way combine is Horner's rule in W_N^{bin} (one complex constant per channel, k_front4).
#include "front_common.h"

namespace mkid {

namespace {

// k_front3 / k_front6 ring plane layout (NW = 4, Q = 256 samples per plane)
__device__ __forceinline__ void ring6_put(uint32_t* hop, int qoff, uint4 v) {
    constexpr int Q = 256;
    const int a = ring3_idx(qoff / 4);
    hop[a] = v.x;
    hop[Q + a] = v.y;
    hop[2 * Q + a] = v.z;
    hop[3 * Q + a] = v.w;
}

struct G6 {
    static constexpr int N = 2048, NW = 4, FW = 4, SPT = 512, BT = FW * 64 + SPT;
    static constexpr int M = N / 2, C = N / 2, T = kPfbTaps, CPT = C / SPT;
    static constexpr int RS = 2 * T + 1;                  // ring slots (hops)
    static constexpr int REG = 576, FB = NW * REG, NB = 2;
    static constexpr size_t off_fbuf = (size_t)RS * M * 4;
    static constexpr size_t off_tw1 = off_fbuf + (size_t)NB * FB * 8;   // W_512^{L k}: [k-1][L]
    static constexpr size_t off_tw2 = off_tw1 + (size_t)7 * 64 * 8;     // W_64^{l k}: [k-1][l]
    static constexpr size_t lds_bytes = off_tw2 + (size_t)7 * 8 * 8;
    static_assert(CPT == 2 && FW * 64 * 4 == M && T == 4, "k_front6 geometry");
    static_assert(2 * lds_bytes <= 160 * 1024, "two workgroups per CU");
};

}  // namespace

#ifdef MKID_XP_STAMPS
#define STAMP6(slot_)                                                                             \
    do {                                                                                          \
        __builtin_amdgcn_sched_barrier(0);                                                        \
        const uint64_t tm_ = __builtin_amdgcn_s_memtime();                                        \
        __builtin_amdgcn_sched_barrier(0);                                                        \
        if (blockIdx.x < 4 && t >= 16 && t < 24 && (threadIdx.x & 63) == 0)                      \
            reinterpret_cast<uint64_t*>(a.phase)[((blockIdx.x * 16 + (threadIdx.x >> 6)) * 8 +   \
                                                  (t - 16)) * 16 + (slot_)] = tm_;                \
    } while (0)
#else
#define STAMP6(slot_) ((void)0)
#endif

// 6 waves per SIMD (two 12-wave workgroups per CU): at most 80 VGPRs
__global__ __launch_bounds__(G6::BT, 6) void k_front6(FrontArgs a) {
    using G = G6;
    constexpr int N = G::N, NW = G::NW, M = G::M, C = G::C, T = G::T, RS = G::RS, CPT = G::CPT;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t* ring = reinterpret_cast<uint32_t*>(smem);
    float2* fbuf = reinterpret_cast<float2*>(smem + G::off_fbuf);
    float2* tw1 = reinterpret_cast<float2*>(smem + G::off_tw1);
    float2* tw2 = reinterpret_cast<float2*>(smem + G::off_tw2);

    const int tid = threadIdx.x;
    const int L = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool xform = wave < G::FW;
    const int rw = xform ? wave : wave - G::FW;

    for (int i = tid; i < 7 * 64; i += G::BT) {
        const int k = i / 64 + 1, l = i % 64;
        double sn, cs;
        sincospi(-2.0 * (double)(l * k) / 512.0, &sn, &cs);
        tw1[i] = make_float2((float)cs, (float)sn);
    }
    for (int i = tid; i < 7 * 8; i += G::BT) {
        const int k = i / 8 + 1, l = i % 8;
        double sn, cs;
        sincospi(-2.0 * (double)(l * k) / 64.0, &sn, &cs);
        tw2[i] = make_float2((float)cs, (float)sn);
    }

    const int64_t k_b = (int64_t)blockIdx.x * a.frames_per_block;
    int64_t k_e = k_b + a.frames_per_block;
    if (k_e > a.K) k_e = a.K;
    if (k_b >= k_e) return;
    const int64_t k_start = k_b - kLpfHist;
    const int nrun = (int)(k_e - k_b);       // even: K and frames_per_block are
    const int nit = nrun + kLpfHist;         // frames from k_start (even)

    if (xform) {
        // ---------------- transform waves: PFB + 512-point sub-FFT w of frame k = k_start + t ---
        const int w = rw;
        const int xt = rw * 64 + L;                          // refill: samples 4 xt .. 4 xt + 3 of a hop
        for (int h = 0; h < 2 * T; ++h) {                    // prologue: hops k_start - 7 .. k_start
            const int64_t hop = k_start - 2 * T + 1 + h;
            ring6_put(ring + (int)(((hop % RS) + RS) % RS) * M, 4 * xt, front_load4<M>(a, hop, xt));
        }
        uint2 tq[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) tq[r] = a.pfbq[NW * (64 * r + L) + w];
        const int la = L & 7, kl = L >> 3;
        const float2* t1 = tw1 + L;               // W_512^{L k} at t1[64 (k - 1)]
        const float2* t2 = tw2 + la;              // W_64^{la k} at t2[8 (k - 1)]
        int rb = (int)((((k_start + 1 - 2 * T) % RS) + RS) % RS);   // slot of hop k - 7
        __syncthreads();
        for (int t = 0; t <= nit; ++t) {
            STAMP6(0);
            if (t < nit) {
                // the hop iteration t + 1 adds: loaded now, written after this wave's sub-FFT
                const uint4 pre = front_load4<M>(a, k_start + t + 1, xt);
                float2* reg = fbuf + (t & 1) * G::FB + w * G::REG;
                float2 v[8];
                uint32_t xr[8][T];
#pragma unroll
                for (int hi = 0; hi < 2; ++hi)
#pragma unroll
                    for (int tau = 0; tau < T; ++tau) {
                        int sl = rb + 2 * tau + hi;
                        sl -= sl >= RS ? RS : 0;
                        const uint32_t* pl = ring + sl * M + w * (M / NW) + 2 * L;
                        const uint2 p01 = *reinterpret_cast<const uint2*>(pl);
                        const uint2 p23 = *reinterpret_cast<const uint2*>(pl + 128);
                        xr[4 * hi + 0][tau] = p01.x;
                        xr[4 * hi + 1][tau] = p01.y;
                        xr[4 * hi + 2][tau] = p23.x;
                        xr[4 * hi + 3][tau] = p23.y;
                    }
#pragma unroll
                for (int r = 0; r < 8; ++r) {
                    const uint32_t i01 = __builtin_amdgcn_perm(xr[r][1], xr[r][0], kPermI);
                    const uint32_t q01 = __builtin_amdgcn_perm(xr[r][1], xr[r][0], kPermQ);
                    const uint32_t i23 = __builtin_amdgcn_perm(xr[r][3], xr[r][2], kPermI);
                    const uint32_t q23 = __builtin_amdgcn_perm(xr[r][3], xr[r][2], kPermQ);
                    int32_t ai = dot2_first(tq[r].x, i01);
                    ai = __builtin_amdgcn_sdot2(as_s2(tq[r].y), as_s2(i23), ai, false);
                    int32_t aq = dot2_first(tq[r].x, q01);
                    aq = __builtin_amdgcn_sdot2(as_s2(tq[r].y), as_s2(q23), aq, false);
                    v[r] = make_float2((float)ai, (float)aq);
                }
                dft<8>(v);
#pragma unroll
                for (int k = 1; k < 8; ++k) v[k] = cmul_pk(v[k], t1[64 * (k - 1)]);
                t1_lds(v, reg, L);
                dft<8>(v);
#pragma unroll
                for (int k = 1; k < 8; ++k) v[k] = cmul_pk(v[k], t2[8 * (k - 1)]);
                float2* t2w = reg + 72 * kl + la;
                const float2* t2r = reg + 72 * kl + 9 * la;
#pragma unroll
                for (int r = 0; r < 8; ++r) t2w[9 * r] = v[r];
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int r = 0; r < 8; ++r) v[r] = t2r[r];
                dft<8>(v);
                __builtin_amdgcn_wave_barrier();
                float2* yw = reg + ((kl + 8 * la) ^ (la << 1));
#pragma unroll
                for (int r = 0; r < 8; ++r) yw[64 * r] = v[r];
                // ring refill: hop k + 1 over hop k - 8 (no reader this iteration)
                int ws = rb + 2 * T;
                ws -= ws >= RS ? RS : 0;
                ring6_put(ring + ws * M, 4 * xt, pre);
                rb += 1;
                rb -= rb >= RS ? RS : 0;
            }
            STAMP6(1);
            __syncthreads();
            STAMP6(2);
        }
    } else {
        // ---------------- select waves: frame k - 1, channels st + SPT q -------------------------
        const int st = rw * 64 + L;
        int cq[CPT];
#pragma unroll
        for (int q = 0; q < CPT; ++q) cq[q] = a.slot_ch ? (int)a.slot_ch[st + G::SPT * q] : st + G::SPT * q;
        float2 tb[CPT];     // W_N^{bin}: X[bin] = ((Y_3 t + Y_2) t + Y_1) t + Y_0
        int yoff[CPT];
#pragma unroll
        for (int q = 0; q < CPT; ++q) {
            const int32_t bin = a.bins[cq[q]];
            double sn, cs;
            sincospi(-2.0 * (double)(bin % N) / N, &sn, &cs);
            tb[q] = make_float2((float)cs, (float)sn);
            yoff[q] = yswz(bin & 511);
        }
        uint64_t gp[13];
#pragma unroll
        for (int m = 0; m < 13; ++m) gp[m] = tap_pair(a.taps.g[2 * m], a.taps.g[2 * m + 1]);
        float2 acc[CPT][13];
#pragma unroll
        for (int q = 0; q < CPT; ++q)
#pragma unroll
            for (int m = 0; m < 13; ++m) acc[q][m] = make_float2(0.f, 0.f);
        float2 ys[CPT];
#pragma unroll
        for (int q = 0; q < CPT; ++q) ys[q] = make_float2(0.f, 0.f);
        int16_t* const raw_run = a.raw + (k_b >> 1) * C;
        float* const phase_run = a.phase ? a.phase + (k_b >> 1) * C : nullptr;
        int lrow = (int)((a.k0 + k_start) & (int64_t)(a.P - 1));
        // z of frame k - 1 (Y buffer b) for both channels
        auto zframe = [&](int b, float2 (&z)[CPT]) {
            const float2* yf = fbuf + b * G::FB;
            const float2* row = a.lo + (lrow & (a.P - 1)) * C;
#pragma unroll
            for (int q = 0; q < CPT; ++q) {
                // per-lane addresses rebuilt in the loop from an opaque channel index (a few VALU)
                // instead of hoisted 64-bit pointers that crowd the 80-register budget
                int cc = cq[q];
                asm volatile("" : "+v"(cc));
                const float2 lo = row[cc];
                const float2* yq = yf + yoff[q];
                float2 X = yq[3 * G::REG];
                X = cmac(yq[2 * G::REG], X, tb[q]);
                X = cmac(yq[G::REG], X, tb[q]);
                X = cmac(yq[0], X, tb[q]);
                z[q] = cmul_pk(X, lo);
            }
            ++lrow;
        };
        __syncthreads();                 // prologue
        [[maybe_unused]] int t = 0;   // iteration (STAMP6)
        STAMP6(3);
        __syncthreads();                 // iteration 0: no frame to select yet
        // iterations (2p + 1, 2p + 2): frame kf = 2p - 24 (accumulate) and 2p - 23 (output)
        for (int p = 0; 2 * p + 2 <= nit; ++p) {
            t = 2 * p + 1;
            STAMP6(3);
            {
                float2 z[CPT];
                zframe(0, z);            // frame kf even was written in iteration 2p: buffer 0
#pragma unroll
                for (int m = 0; m < 13; ++m)
#pragma unroll
                    for (int q = 0; q < CPT; ++q) acc[q][m] = fma_tap<1>(gp[m], z[q], acc[q][m]);
            }
            STAMP6(4);
            __syncthreads();
            t = 2 * p + 2;
            STAMP6(5);
            {
                float2 z[CPT];
                zframe(1, z);
                float2 y[CPT];
#pragma unroll
                for (int q = 0; q < CPT; ++q) y[q] = fma_tap<0>(gp[0], z[q], acc[q][0]);
#pragma unroll
                for (int m = 0; m < 12; ++m)
#pragma unroll
                    for (int q = 0; q < CPT; ++q) acc[q][m] = fma_tap<0>(gp[m + 1], z[q], acc[q][m + 1]);
#pragma unroll
                for (int q = 0; q < CPT; ++q) acc[q][12] = make_float2(0.f, 0.f);
                const int kf = 2 * p - kLpfHist + 1;
                if (kf > 0 && kf < nrun) {
                    const int jr = (kf - 1) >> 1;
#pragma unroll
                    for (int q = 0; q < CPT; ++q) {
                        int c = cq[q];
                        asm volatile("" : "+v"(c));
                        ys[q].x += y[q].x;
                        ys[q].y += y[q].y;
                        const float ph = phase_atan2(y[q].y - a.qc[c], y[q].x - a.ic[c]);
                        int qv = __float2int_rn(ph * 8192.0f);
                        qv = qv < -25736 ? -25736 : (qv > 25736 ? 25736 : qv);
#ifndef MKID_XP_STAMPS   // the timing build keeps its stamps in the phase buffer
                        if (phase_run) (phase_run + jr * C)[c] = ph;
#endif
                        (raw_run + jr * C)[c] = (int16_t)qv;
                        if (c == a.iq_ch && a.iqtap) {
                            a.iqtap[2 * ((k_b >> 1) + jr)] = iq16(y[q].x);
                            a.iqtap[2 * ((k_b >> 1) + jr) + 1] = iq16(y[q].y);
                        }
                    }
                }
            }
            STAMP6(6);
            __syncthreads();
        }
        if (a.ysum)
#pragma unroll
            for (int q = 0; q < CPT; ++q) ysum_add(a.ysum, cq[q], ys[q].x, ys[q].y);
    }
}

hipError_t launch_front6(const FrontArgs& a0, hipStream_t s) {
    using G = G6;
    static std::atomic<uint64_t> attr_mask{0};
    hipError_t e = ensure_lds_attr(attr_mask, (const void*)k_front6, (int)G::lds_bytes);
    if (e != hipSuccess) return e;
    FrontArgs a = a0;
    if (a.K <= 0) return hipSuccess;
    // two runs per CU (two resident workgroups), runs of <= 2048 frames
    const int64_t ncu = a.ncu > 0 ? a.ncu : 256;
    int64_t fpb = a.K / (2 * ncu);
    fpb = fpb < 64 ? 64 : (fpb > 2048 ? 2048 : fpb);
    fpb = (fpb + 1) / 2 * 2;
    a.frames_per_block = fpb;
    const int64_t blocks = (a.K + fpb - 1) / fpb;
    hipLaunchKernelGGL(k_front6, dim3((unsigned)blocks), dim3(G::BT), G::lds_bytes, s, a);
    return hipGetLastError();
}

}  // namespace mkid
