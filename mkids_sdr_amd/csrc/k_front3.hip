// Fused front end k_front3, the default at N = 512 / 1024 / 2048 (configs 2, 3/4): the PFB, the
// in-wave 512-point sub-FFTs, the bin-select combine, DDC, low-pass and phase, with the waves of a
// workgroup specialised into transform and select roles.
#include "front_common.h"

namespace mkid {

namespace {
// k_front3 ring plane layout (NW = 4, Q = 256 samples per plane): samples qoff..qoff+3 of a hop go
// to planes 0..3 at plane index qoff / 4, paired (ring3_idx). The refill's ds_write_b32 become
// 2-way bank conflicts, which cost no extra cycles for ds_write_b32 (MI355X_MICROARCH.md §LDS).
[[maybe_unused]] __device__ __forceinline__ void ring3_put(uint32_t* hop, int qoff, uint4 v) {
    constexpr int Q = 256;
    const int a = ring3_idx(qoff / 4);
    hop[a] = v.x;
    hop[Q + a] = v.y;
    hop[2 * Q + a] = v.z;
    hop[3 * Q + a] = v.w;
}
}  // namespace
// Why specialise: when every wave runs the FFT phase and then the select phase with a barrier
// between them (the round-2 design, history in DESIGN.md Appendix A), a SIMD idles whenever all its
// waves wait on LDS (ring reads, the select's bin-indexed reads) or on the barrier. Here waves 0-7 only transform
// (2 frames per iteration, one 512-point sub-FFT each) and waves 8-15 only select / mix / low-pass /
// phase (two channels per thread), one iteration behind, on a double-buffered Y: each SIMD holds
// two FFT and two select waves whose LDS waits and VALU bursts interleave, one barrier per
// iteration.
//   ring  RS = 2T - 1 + 2F hops: iteration t reads hops k-7 .. k+1 (frames k, k+1) while its
//         FFT waves write hops k+2, k+3 (prefetched at the loop top) over hops k-9, k-8
//   Y     [2][F][NW][576] float2, iteration t writes buffer t & 1, its select reads (t - 1) & 1
// Registers: the FFT path holds the PFB taps and the 512-point sub-FFT, the select path two
// channels' low-pass state; branches are wave-uniform, so the two live sets do not add up.
// Measured and dropped: LDS progress words instead of the barrier on three Y
// buffers (+5.6 %), roles alternating by age on each SIMD (+2.6 %), issue priority for either
// group or for the younger wave of a pair (zero-sum), non-temporal raw / phase stores (+1.3 %);
// round 4: a pair ring ((x[s], x[s+2]) pair words built once per sample at refill, -8.5 % VALU
// instructions: neutral) and buffer-descriptor select I/O (+2.6 %), commit 21e0b7c; 4 transform
// waves each computing sub-FFT w of both frames, interleaved (+17 %), commit eb8fb42; two
// 768-thread workgroups per CU at one frame per iteration (k_front6, +25 %), commit ac8fe74.

// Geometry per N. N = 2048 (config 3/4): 8 transform waves (4 sub-FFTs x 2 frames) + 8 select
// waves (2 channels per thread), one workgroup per CU. N = 1024 (round 5): 8
// transform waves (2 sub-FFTs x 4 frames) + 8 select waves (1 channel per thread), one workgroup
// per CU. N = 512 (config 2, round 4): 4 transform waves (the 512-point FFT of each of 4 frames) +
// 4 select waves (1 channel per thread), two workgroups per CU.
#ifndef MKID_F3_PF2_N
#define MKID_F3_PF2_N 512
#endif
template <int N>
struct G3 {
    static constexpr int NW = N / 512;                 // sub-FFTs per frame
    static constexpr int F = N == 2048 ? 2 : 4;        // frames per iteration
    static constexpr int FW = F * NW;                  // transform waves (one sub-FFT each)
    static constexpr int SPT = N == 512 ? 256 : 512;   // select threads
    static constexpr int BT = FW * 64 + SPT;
    static constexpr int M = N / 2, C = N / 2, T = kPfbTaps;
    static constexpr int CPT = C / SPT;                // channels per select thread
    static constexpr int RS = 2 * T - 1 + 2 * F;       // ring slots (hops)
    static constexpr int REG = 576;
    static constexpr int FB = NW * REG;
    static constexpr size_t off_fbuf = (size_t)RS * M * 4;
    static constexpr int NB = 2;                       // Y buffers
    static constexpr size_t off_tw1 = off_fbuf + (size_t)NB * F * FB * 8;
    static constexpr size_t off_tw2 = off_tw1 + (size_t)7 * 64 * 8;
    static constexpr size_t lds_bytes = off_tw2 + (size_t)7 * 8 * 8;
    static constexpr int WG_PER_CU = 16 * 64 / BT;     // 16 waves per CU
    // ring prefetch two iterations deep (round 6): N = 512 -2.8 ... -5.8 % in three same-box A/Bs;
    // N = 1024 +1 %, N = 2048 +25 % (profiles/r06/r06{q,x,y}_kbench_*_pf2.log)
    static constexpr bool PF2 = N == MKID_F3_PF2_N;
    static_assert((N == 2048 || N == 1024 || N == 512) && F * M == FW * 64 * 4 && C == SPT * CPT, "k_front3 geometry");
    static_assert(lds_bytes * WG_PER_CU <= 160 * 1024, "LDS");
};

// ring plane layout for any NW (paired planes of Q = M / NW = 256 samples): samples qoff..qoff+3 of
// a hop (qoff a multiple of 4) go to plane o mod NW at plane index o / NW
template <int NW>
__device__ __forceinline__ void ring3_put_nw(uint32_t* hop, int qoff, uint4 v) {
    if constexpr (NW == 4) {
        ring3_put(hop, qoff, v);
    } else if constexpr (NW == 2) {
        constexpr int Q = 256;
        const int a = ring3_idx(qoff / 2);   // plane indices qoff / 2 and qoff / 2 + 1 (at a + 2)
        hop[a] = v.x;
        hop[Q + a] = v.y;
        hop[a + 2] = v.z;
        hop[Q + a + 2] = v.w;
    } else {
        static_assert(NW == 1, "ring layout");
        const int a = ring3_idx(qoff);
        hop[a] = v.x;
        hop[a + 2] = v.y;
        hop[a + 4] = v.z;
        hop[a + 6] = v.w;
    }
}

#ifdef MKID_XP_STAMPS
#define STAMP3(slot_)                                                                             \
    do {                                                                                          \
        __builtin_amdgcn_sched_barrier(0);                                                        \
        const uint64_t tm_ = __builtin_amdgcn_s_memtime();                                        \
        __builtin_amdgcn_sched_barrier(0);                                                        \
        if (blockIdx.x < 4 && t >= 8 && t < 16 && (threadIdx.x & 63) == 0)                        \
            reinterpret_cast<uint64_t*>(a.phase)[((blockIdx.x * 16 + (threadIdx.x >> 6)) * 8 +   \
                                                  (t - 8)) * 16 + (slot_)] = tm_;                 \
    } while (0)
#else
#define STAMP3(slot_) ((void)0)
#endif

template <int N>
__global__ __launch_bounds__(G3<N>::BT, 4) void k_front3(FrontArgs a) {   // 16 waves per CU
    using G = G3<N>;
    constexpr int NW = G::NW, M = G::M, C = G::C, T = G::T, RS = G::RS, F = G::F, CPT = G::CPT;
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
    const int nrun = (int)(k_e - k_b);
    const int nit = (nrun + kLpfHist + F - 1) / F;    // iterations of F frames from k_start

    if (xform) {
        // ---------------- transform waves: PFB + 512-point sub-FFT of (frame slot, w) ----------
        const int slot = rw / NW, w = rw % NW;
        const int xt = rw * 64 + L;                            // thread index among the transform waves
        const int qh = (xt * 4) / M, qoff = (xt * 4) % M;      // this thread's ring write
        {   // prologue: hops k_start-2T+1 .. k_start+F-1
            const int64_t h0 = k_start - 2 * T + 1;
            for (int g = 0; g < 2 * T - 1 + F; g += 2) {
                const int64_t hop = h0 + g + qh;
                if (hop > h0 + 2 * T - 2 + F) continue;
                const uint4 v = front_load4<M>(a, h0 + g, xt);
                ring3_put_nw<NW>(ring + (int)(((hop % RS) + RS) % RS) * M, qoff, v);
            }
        }
        uint2 tq[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) tq[r] = a.pfbq[NW * (64 * r + L) + w];
        // the taps are complete before the loop: otherwise the loop's waits on them (vmcnt counts
        // retire in order) also wait on each iteration's ring prefetch, exposing its HBM latency
        // (N = 1024: -3.6 %; N = 512, scheduled max-ILP: +3 %, left to the scheduler there;
        // profiles/r05/r05al_kbench_{c2,512}_tq.json)
        if constexpr (N != 512) {
#pragma unroll
            for (int r = 0; r < 8; ++r) asm volatile("" : "+v"(tq[r].x), "+v"(tq[r].y));
        }
        const int la = L & 7, kl = L >> 3;
        const float2* t1 = tw1 + L;
        const float2* t2 = tw2 + la;
        int rb = (int)((((k_start + 1 - 2 * T) % RS) + RS) % RS);   // slot of hop k - 2T + 1
        __syncthreads();
        // the lane's 14 twiddles are the same every iteration: held in VGPRs (the transform path
        // has registers to spare), 14 fewer LDS reads per sub-FFT on an LDS that is ~60 % busy
        float2 w1[7], w2[7];
#pragma unroll
        for (int k = 1; k < 8; ++k) {
            w1[k - 1] = t1[64 * (k - 1)];
            w2[k - 1] = t2[8 * (k - 1)];
            asm volatile("" : "+v"(w1[k - 1].x), "+v"(w1[k - 1].y), "+v"(w2[k - 1].x), "+v"(w2[k - 1].y));
        }
        // the transform work of iteration t: ring reads, PFB, sub-FFT, Y write
        auto transform = [&](int t) __attribute__((always_inline)) {
            float2* reg = fbuf + ((t % G::NB) * F + slot) * G::FB + w * G::REG;
            int sb = rb + slot;
            sb -= sb >= RS ? RS : 0;
            float2 v[8];
            uint32_t xr[8][T];
#pragma unroll
            for (int hi = 0; hi < 2; ++hi)
#pragma unroll
                for (int tau = 0; tau < T; ++tau) {
                    int sl = sb + 2 * tau + hi;
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
                uint32_t x4[T];
#pragma unroll
                for (int tau = 0; tau < T; ++tau) x4[tau] = xr[r][tau];
                const uint32_t i01 = __builtin_amdgcn_perm(x4[1], x4[0], kPermI);
                const uint32_t q01 = __builtin_amdgcn_perm(x4[1], x4[0], kPermQ);
                const uint32_t i23 = __builtin_amdgcn_perm(x4[3], x4[2], kPermI);
                const uint32_t q23 = __builtin_amdgcn_perm(x4[3], x4[2], kPermQ);
                int32_t ai = dot2_first(tq[r].x, i01);
                ai = __builtin_amdgcn_sdot2(as_s2(tq[r].y), as_s2(i23), ai, false);
                int32_t aq = dot2_first(tq[r].x, q01);
                aq = __builtin_amdgcn_sdot2(as_s2(tq[r].y), as_s2(q23), aq, false);
                v[r] = make_float2((float)ai, (float)aq);
            }
            dft<8>(v);
#pragma unroll
            for (int k = 1; k < 8; ++k) v[k] = cmul_pk(v[k], w1[k - 1]);
            t1_lds(v, reg, L);
            dft<8>(v);
#pragma unroll
            for (int k = 1; k < 8; ++k) v[k] = cmul_pk(v[k], w2[k - 1]);
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
        };
        if constexpr (!G::PF2) {
            for (int t = 0; t <= nit; ++t) {
                STAMP3(0);
                if (t < nit) {
                    const int kr = -kLpfHist + F * t;
                    // the hops iteration t + 1 adds: loaded now, written after this wave's PFB
                    const uint4 pre = front_load4<M>(a, k_b + kr + F, xt);
                    transform(t);
                    // ring refill: hops k+F .. k+2F-1 over hops k-2T-1 .. (no reader this iteration)
                    int ws = rb + 2 * T - 1 + F + qh;
                    ws -= ws >= RS ? RS : 0;
                    ws -= ws >= RS ? RS : 0;
                    ring3_put_nw<NW>(ring + ws * M, qoff, pre);
                    rb += F;
                    rb -= rb >= RS ? RS : 0;
                }
                STAMP3(1);
                __syncthreads();
                STAMP3(2);
            }
        } else {
            // the prefetch two iterations deep, unrolled by 2 so that the two loads in flight sit in
            // fixed registers and the wait before each refill leaves the newer one outstanding
            // (vmcnt(1)); the loads are unconditional (past the run they read unused words)
            auto iter = [&](int t, const Load4& use, Load4& fill) __attribute__((always_inline)) {
                STAMP3(0);
                const int kr = -kLpfHist + F * t;
                fill = front_load4_nb<M>(a, k_b + kr + 2 * F, xt);   // the hops iteration t + 2 adds
                transform(t);
                int ws = rb + 2 * T - 1 + F + qh;   // the ring refill, as above
                ws -= ws >= RS ? RS : 0;
                ws -= ws >= RS ? RS : 0;
                ring3_put_nw<NW>(ring + ws * M, qoff, use.past ? make_uint4(0, 0, 0, 0) : use.v);
                rb += F;
                rb -= rb >= RS ? RS : 0;
                STAMP3(1);
                __syncthreads();
                STAMP3(2);
            };
            Load4 pa = front_load4_nb<M>(a, k_b - kLpfHist + F, xt), pb;
            int t = 0;
            for (; t + 1 < nit; t += 2) {
                iter(t, pa, pb);
                iter(t + 1, pb, pa);
            }
            if (t < nit) iter(t, pa, pb);
            STAMP3(0);   // t = nit: the select waves' last iteration
            STAMP3(1);
            __syncthreads();
            STAMP3(2);
        }
    } else {
        // ---------------- select waves: channels st + SPT q, one iteration behind ---------------
        const int st = rw * 64 + L;
        float2 tl[CPT][NW > 1 ? NW - 1 : 1];
        int yoff[CPT];
        float2 ncen[CPT], cor[CPT];   // -c' and r of the centred low-pass (mkid_internal.h Centring)
        // channel of (thread, q): a host-chosen order (mkid_api.hip slot_order) that puts the 32
        // channels each half-wave reads per instruction on distinct LDS bank pairs of Y, each
        // wave keeping its own 128 channels (stores and LO loads stay within 2-4 lines)
        int cq[CPT];
#pragma unroll
        for (int q = 0; q < CPT; ++q) cq[q] = a.slot_ch ? (int)a.slot_ch[st + G::SPT * q] : st + G::SPT * q;
#pragma unroll
        for (int q = 0; q < CPT; ++q) {
            const int c = cq[q];
            const int32_t bin = a.bins[c];
#pragma unroll
            for (int u = 1; u < NW; ++u) {
                double sn, cs;
                sincospi(-2.0 * (double)((u * bin) % N) / N, &sn, &cs);
                tl[q][u - 1] = make_float2((float)cs, (float)sn);
            }
            yoff[q] = yswz(bin & 511);
            ncen[q] = a.cen.ncen[c];
            cor[q] = a.cen.cor[c];
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
        __syncthreads();
        for (int t = 0; t <= nit; ++t) {
            STAMP3(3);
            if (t > 0) {
                const int kr = -kLpfHist + F * (t - 1);
                float2 lov[F][CPT];
#pragma unroll
                for (int f = 0; f < F; ++f) {
                    const float2* row = a.lo + ((lrow + f) & (a.P - 1)) * C;
#pragma unroll
                    for (int q = 0; q < CPT; ++q) lov[f][q] = row[cq[q]];
                }
                lrow += F;
#pragma unroll
                for (int f = 0; f < F; ++f) {
                    const int kf = kr + f;
                    const float2* yf = fbuf + (((t - 1) % G::NB) * F + f) * G::FB;
                    float2 z[CPT];
#pragma unroll
                    for (int q = 0; q < CPT; ++q) {
                        float2 X = yf[yoff[q]];
#pragma unroll
                        for (int u = 1; u < NW; ++u) X = cmac(X, tl[q][u - 1], yf[yoff[q] + u * G::REG]);
                        z[q] = cmul_add_pk(X, lov[f][q], ncen[q]);   // z - c'
                    }
                    if ((f & 1) == 0) {
#pragma unroll
                        for (int m = 0; m < 13; ++m)
#pragma unroll
                            for (int q = 0; q < CPT; ++q) acc[q][m] = fma_tap<1>(gp[m], z[q], acc[q][m]);
                    } else {
                        float2 y[CPT];
#pragma unroll
                        for (int q = 0; q < CPT; ++q) y[q] = fma_tap<0>(gp[0], z[q], acc[q][0]);
#pragma unroll
                        for (int m = 0; m < 12; ++m)
#pragma unroll
                            for (int q = 0; q < CPT; ++q) acc[q][m] = fma_tap<0>(gp[m + 1], z[q], acc[q][m + 1]);
#pragma unroll
                        for (int q = 0; q < CPT; ++q) acc[q][12] = make_float2(0.f, 0.f);
                        if (kf > 0 && kf < nrun) {
                            const int jr = (kf - 1) >> 1;
#pragma unroll
                            for (int q = 0; q < CPT; ++q) {
                                const int c = cq[q];
                                ys[q].x += y[q].x;
                                ys[q].y += y[q].y;
                                const float ph = phase_atan2(y[q].y + cor[q].y, y[q].x + cor[q].x);
                                int qv = __float2int_rn(ph * 8192.0f);
                                qv = qv < -25736 ? -25736 : (qv > 25736 ? 25736 : qv);
                                // plain stores: with the slot order a wave's store covers its 64
                                // channels within 2 (raw) or 4 (phase) lines, merged in L2
#ifndef MKID_XP_STAMPS   // the timing build keeps its stamps in the phase buffer
                                if (phase_run) (phase_run + jr * C)[c] = ph;
#endif
                                (raw_run + jr * C)[c] = (int16_t)qv;
                                if (c == a.iq_ch && a.iqtap) {
                                    a.iqtap[2 * ((k_b >> 1) + jr)] = iq16(y[q].x + a.cen.tap_off.x);
                                    a.iqtap[2 * ((k_b >> 1) + jr) + 1] = iq16(y[q].y + a.cen.tap_off.y);
                                }
                            }
                        }
                    }
                }
            }
            STAMP3(4);
            __syncthreads();
            STAMP3(5);
        }
        if (a.ysum)
#pragma unroll
            for (int q = 0; q < CPT; ++q) ysum_add(a.ysum, cq[q], ys[q].x, ys[q].y);
    }
}

template <int N>
static hipError_t launch_front3_n(const FrontArgs& a0, hipStream_t s) {
    using G = G3<N>;
    static std::atomic<uint64_t> attr_mask{0};
    hipError_t e = ensure_lds_attr(attr_mask, (const void*)k_front3<N>, (int)G::lds_bytes);
    if (e != hipSuccess) return e;
    FrontArgs a = a0;
    if (a.K <= 0) return hipSuccess;
    const int64_t ncu = a.ncu > 0 ? a.ncu : 256;
    int64_t fpb = a.K / (ncu * G::WG_PER_CU);    // one run per resident workgroup
    fpb = fpb < 64 ? 64 : (fpb > 4096 ? 4096 : fpb);
    fpb = (fpb + G::F - 1) / G::F * G::F;
    a.frames_per_block = fpb;
    const int64_t blocks = (a.K + fpb - 1) / fpb;
    hipLaunchKernelGGL(k_front3<N>, dim3((unsigned)blocks), dim3(G::BT), G::lds_bytes, s, a);
    return hipGetLastError();
}

#ifdef MKID_F3_N
// One geometry per object (Makefile: k_front3_<N>.o), so that each takes scheduler flags of its
// own (F3_FLAGS_<N>); the N = 2048 object also holds the dispatch.
hipError_t launch_front3_512(const FrontArgs& a, hipStream_t s);
hipError_t launch_front3_1024(const FrontArgs& a, hipStream_t s);
hipError_t launch_front3_2048(const FrontArgs& a, hipStream_t s);
#define MKID_F3_CAT2(a, b) a##b
#define MKID_F3_CAT(a, b) MKID_F3_CAT2(a, b)
hipError_t MKID_F3_CAT(launch_front3_, MKID_F3_N)(const FrontArgs& a, hipStream_t s) {
    return launch_front3_n<MKID_F3_N>(a, s);
}
#if MKID_F3_N == 2048
hipError_t launch_front3(int N, const FrontArgs& a, hipStream_t s) {
    switch (N) {
        case 2048: return launch_front3_2048(a, s);
        case 1024: return launch_front3_1024(a, s);
        case 512: return launch_front3_512(a, s);
        default: return hipErrorInvalidValue;
    }
}
#endif
#else
hipError_t launch_front3(int N, const FrontArgs& a, hipStream_t s) {
    switch (N) {
        case 2048: return launch_front3_n<2048>(a, s);
        case 1024: return launch_front3_n<1024>(a, s);
        case 512: return launch_front3_n<512>(a, s);
        default: return hipErrorInvalidValue;
    }
}
#endif

}  // namespace mkid
