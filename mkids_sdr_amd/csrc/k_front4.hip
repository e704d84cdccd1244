// Fused front end for N = 4096 (2048 channels, BASELINE config 5): K1-K6 in one pass over the ADC
// stream, the complex baseband never leaving the chip (the split path stages it through HBM at
// +16 B per ADC sample). Same FFT scheme as k_front2.hip (decimation in time by NW = 8 sub-FFTs of
// 512 points, each computed inside one wave, one cross-wave exchange per frame), re-balanced for
// a 2048-channel frame:
//
//  * a 1024-thread workgroup (16 waves, 4 per SIMD, <= 128 VGPRs) walks its run FPB = 2 frames per
//    iteration; wave (s, w) computes sub-FFT w of frame s, thread t then owns the two channels
//    t + 1024 q (q = 0, 1) in the select / DDC / low-pass / phase stage. (512-thread workgroups, 8
//    waves, 2 per SIMD, 4 channels per thread, no spills, were 7 % slower: two waves per SIMD cannot
//    hide the barrier phases; the 1024-thread build spills ~21 loop-invariant dwords and still wins);
//  * the PFB taps of a wave's points are the same every frame, so they live in VGPRs (8 int16
//    quads per lane) and the LDS holds only the ADC ring (9 hops, 72 KiB), the Y buffers of the two
//    frames (72 KiB) and the two twiddle tables: 151.5 KiB of the CU's 160 KiB;
//  * X[bin] = sum_w W_N^{w bin} Y_w[bin mod 512] is evaluated as two 4-term Horner chains in
//    W_N^{bin} joined by W_N^{4 bin} (two complex constants per channel instead of seven);
//  * the decimating low-pass folds its accumulator shift into the output frame's FMAs.
// Index maps and LDS layouts are those of k_front2.hip at NW = 8 (tools/front2_layouts.py).
#include "front_common.h"

#ifdef MKID_XP_STAMPS
// timing-only build: lane 0 of every wave of workgroups 0-3 stamps s_memtime at 6 points of
// iterations 8..15 into a.phase (tools/stamps4.py); the phase output of that build is garbage
#define STAMP4(slot_)                                                                             \
    do {                                                                                          \
        __builtin_amdgcn_sched_barrier(0);                                                        \
        const uint64_t tm_ = __builtin_amdgcn_s_memtime();                                        \
        __builtin_amdgcn_sched_barrier(0);                                                        \
        if (blockIdx.x < 4 && it_ >= 8 && it_ < 16 && (threadIdx.x & 63) == 0)                   \
            reinterpret_cast<uint64_t*>(a.phase)[((blockIdx.x * 16 + (threadIdx.x >> 6)) * 8 +   \
                                                  (it_ - 8)) * 8 + (slot_)] = tm_;                \
    } while (0)
#else
#define STAMP4(slot_) ((void)0)
#endif

namespace mkid {

namespace {

struct G4 {
    static constexpr int N = 4096, NW = 8, FPB = 2, BT = 1024, CPT = 2048 / BT;
    static constexpr int SPW = FPB * NW * 64 / BT;     // sub-FFTs per wave per iteration
    static constexpr int SPT = FPB * (N / 2) / BT;     // ring-refill samples per thread (8 or 4)
    static constexpr int M = N / 2, C = N / 2, T = kPfbTaps;
    static constexpr int RS = 2 * T - 1 + FPB;         // ring slots (hops)
    static constexpr int Q = M / NW;                   // samples per hop plane
    static constexpr int REG = 576;                    // float2 per (frame, wave) region
    static constexpr int FB = NW * REG;                // float2 per frame
    static constexpr int HIST = (2 * T - 1 + kLpfHist) * M;
    static constexpr size_t off_fbuf = (size_t)RS * M * 4;
    static constexpr size_t off_tw1 = off_fbuf + (size_t)FPB * FB * 8;  // W_512^{L k}: [k-1][L]
    static constexpr size_t off_tw2 = off_tw1 + (size_t)7 * 64 * 8;    // W_64^{l k}: [k-1][l]
    static constexpr size_t lds_bytes = off_tw2 + (size_t)7 * 8 * 8;
    static_assert(BT * CPT == C && SPW * BT == FPB * NW * 64 && (SPT == 8 || SPT == 4), "geometry");
    static_assert(lds_bytes <= 160 * 1024, "LDS");
};

// the SPT samples (SPT*4 bytes) this thread contributes to the FPB hops starting at first_hop
__device__ __forceinline__ void load8(const FrontArgs& a, int64_t first_hop, int tid, uint4& v0, uint4& v1) {
    constexpr int SPT = G4::SPT;
    const int64_t s0 = first_hop * G4::M + (int64_t)tid * SPT;
    if (s0 >= a.K * G4::M) {
        v0 = v1 = make_uint4(0, 0, 0, 0);
        return;
    }
    if (s0 >= -a.avail) {
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 p = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a.x + s0));
        v0 = make_uint4(p.x, p.y, p.z, p.w);
        if constexpr (SPT == 8) {
            const u32x4 q = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a.x + s0 + 4));
            v1 = make_uint4(q.x, q.y, q.z, q.w);
        }
        return;
    }
    const uint32_t* h = a.xhist + (s0 + a.avail + G4::HIST);
    v0 = *reinterpret_cast<const uint4*>(h);
    if constexpr (SPT == 8) v1 = *reinterpret_cast<const uint4*>(h + 4);
}

// samples qoff..qoff+7 of a hop (qoff a multiple of 8) into the permuted hop layout: sample o at
// (o % 8) Q + o / 8, i.e. one dword in each of the 8 planes (consecutive lanes, consecutive dwords)
// (SPT = 4: samples qoff..qoff+3 go to planes qoff % 8 .. + 3; lanes 2k, 2k+1 share a bank, 2-way)
// plane index i at ring3_idx(i) (paired planes), so the PFB reads points r, r + 1 of a lane with
// one ds_read_b64
__device__ __forceinline__ void ring_put8(uint32_t* hop, int qoff, uint4 v0, uint4 v1) {
    constexpr int Q = G4::Q;
    uint32_t* p = hop + (qoff % 8) * Q + ring3_idx(qoff / 8);
    p[0] = v0.x; p[Q] = v0.y; p[2 * Q] = v0.z; p[3 * Q] = v0.w;
    if constexpr (G4::SPT == 8) {
        p[4 * Q] = v1.x; p[5 * Q] = v1.y; p[6 * Q] = v1.z; p[7 * Q] = v1.w;
    }
}

}  // namespace

__global__ __launch_bounds__(G4::BT, G4::BT / 256) void k_front4(FrontArgs a) {
    using G = G4;
    constexpr int NW = G::NW, M = G::M, C = G::C, T = G::T, RS = G::RS, FPB = G::FPB, CPT = G::CPT;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t* ring = reinterpret_cast<uint32_t*>(smem);
    float2* fbuf = reinterpret_cast<float2*>(smem + G::off_fbuf);
    float2* tw1 = reinterpret_cast<float2*>(smem + G::off_tw1);
    float2* tw2 = reinterpret_cast<float2*>(smem + G::off_tw2);

    const int tid = threadIdx.x;
    const int L = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int w = wave % NW;                   // this wave's sub-FFT
    const int slot0 = (wave / NW) * G::SPW;    // its first frame slot (SPW consecutive slots)


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
    // PFB tap quads of this lane's points NW (64 r + L) + w, r = 0..7 (fixed for every frame)
    uint2 tq[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) tq[r] = a.pfbq[NW * (64 * r + L) + w];

    // select constants of channels c_q = tid + 512 q
    float2 tb[CPT], tb4[CPT];   // W_N^{bin}, W_N^{4 bin}
    int yoff[CPT];
    float ic[CPT], qc[CPT];
#pragma unroll
    for (int q = 0; q < CPT; ++q) {
        const int c = tid + G::BT * q;
        const int32_t bin = a.bins[c];
        double sn, cs;
        sincospi(-2.0 * (double)bin / G::N, &sn, &cs);
        tb[q] = make_float2((float)cs, (float)sn);
        sincospi(-2.0 * (double)((4 * bin) % G::N) / G::N, &sn, &cs);
        tb4[q] = make_float2((float)cs, (float)sn);
        yoff[q] = yswz(bin & 511);
        ic[q] = a.ic[c];
        qc[q] = a.qc[c];
    }

    // low-pass taps as 13 uniform pairs (g_{2m}, g_{2m+1}) for packed FMAs (fma_tap)
    uint64_t gp[13];
#pragma unroll
    for (int m = 0; m < 13; ++m) gp[m] = tap_pair(a.taps.g[2 * m], a.taps.g[2 * m + 1]);

    const int64_t k_b = (int64_t)blockIdx.x * a.frames_per_block;
    int64_t k_e = k_b + a.frames_per_block;
    if (k_e > a.K) k_e = a.K;
    if (k_b >= k_e) return;
    const int64_t k_start = k_b - kLpfHist;
    int16_t* const raw_run = a.raw + (k_b >> 1) * C;
    float* const phase_run = a.phase ? a.phase + (k_b >> 1) * C : nullptr;

    const int qh = (tid * G::SPT) / M, qoff = (tid * G::SPT) % M;  // this thread's ring write
    {   // prologue: hops k_start-2T+1 .. k_start+FPB-1 -> ring (slot = hop mod RS)
        const int64_t h0 = k_start - 2 * T + 1;
        for (int g = 0; g < RS; g += FPB) {
            const int64_t hop = h0 + g + qh;
            if (hop > h0 + RS - 1) continue;
            uint4 v0, v1;
            load8(a, h0 + g, tid, v0, v1);
            ring_put8(ring + (int)(((hop % RS) + RS) % RS) * M, qoff, v0, v1);
        }
    }
    __syncthreads();

    float2 acc[CPT][13];
#pragma unroll
    for (int q = 0; q < CPT; ++q)
#pragma unroll
        for (int m = 0; m < 13; ++m) acc[q][m] = make_float2(0.f, 0.f);
    float2 ys[CPT];
#pragma unroll
    for (int q = 0; q < CPT; ++q) ys[q] = make_float2(0.f, 0.f);

    int rb = (int)((((k_start + 1 - 2 * T) % RS) + RS) % RS);
    int lrow = (int)((a.k0 + k_start) & (int64_t)(a.P - 1));
    const int nrun = (int)(k_e - k_b);
    const int la = L & 7, kl = L >> 3;
    const float2* t1 = tw1 + L;
    const float2* t2 = tw2 + la;

#ifdef MKID_XP_STAMPS
    int it_ = 0;
#endif
    for (int kr = -kLpfHist; kr < nrun; kr += FPB) {
#ifdef MKID_XP_STAMPS
        ++it_;
#endif
        STAMP4(0);
        // this iteration's ring refill (its oldest FPB hops, written after the FFT barrier):
        // loaded here, so the 8 registers live only through the FFT phase and no ring load is
        // outstanding in the select phase (vmcnt waits are in issue order)
        uint4 pre0 = make_uint4(0, 0, 0, 0), pre1 = pre0;
        load8(a, k_b + kr + FPB, tid, pre0, pre1);
        // LO rows of the iteration's frames: scalar row base + 32-bit lane offsets (global_load
        // with an SGPR base). Loaded here (live across the FFT) with 512-thread workgroups; with
        // 1024 (2 channels per thread, 128 VGPRs) after the FFT, where the registers are free
        float2 lov[FPB][CPT];
        auto load_lo = [&]() {
#pragma unroll
            for (int f = 0; f < FPB; ++f) {
                const char* row = reinterpret_cast<const char*>(a.lo + ((lrow + f) & (a.P - 1)) * C);
#pragma unroll
                for (int q = 0; q < CPT; ++q)
                    lov[f][q] = *reinterpret_cast<const float2*>(row + (uint32_t)(tid + G::BT * q) * 8u);
            }
        };
        if constexpr (G::BT == 512) load_lo();

#pragma unroll
        for (int si = 0; si < G::SPW; ++si) {
            const int sl0 = slot0 + si;
            float2* reg = fbuf + sl0 * G::FB + w * G::REG;
            // ---- PFB: points NW (64 r + L) + w of frame kb + sl0 ----
            int sb = rb + sl0;
            sb -= sb >= RS ? RS : 0;
            float2 v[8];
            uint32_t xo[T];   // the odd point's samples (paired planes)
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const int hi = r >> 2;
                uint32_t x4[T];
                if ((r & 1) == 0) {
#pragma unroll
                    for (int tau = 0; tau < T; ++tau) {
                        int s = sb + 2 * tau + hi;
                        s -= s >= RS ? RS : 0;
                        const uint2 p = *reinterpret_cast<const uint2*>(ring + s * M + w * G::Q + 128 * ((r & 3) >> 1) + 2 * L);
                        x4[tau] = p.x;
                        xo[tau] = p.y;
                    }
                } else {
#pragma unroll
                    for (int tau = 0; tau < T; ++tau) x4[tau] = xo[tau];
                }
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
            // ---- stage 1 + W_512^{L k}, T1, stage 2 + W_64^{la k}, T2 (own region), stage 3 ----
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
        }
        STAMP4(1);
        __syncthreads();  // Y of both frames visible; every ring read of this iteration done
        STAMP4(2);
        if constexpr (G::BT != 512) load_lo();

        {   // ring refill for the next iteration (its oldest FPB hops), prefetch one further
            int ws = rb + qh;
            ws -= ws >= RS ? RS : 0;
            ring_put8(ring + ws * M, qoff, pre0, pre1);
            rb += FPB;
            rb -= rb >= RS ? RS : 0;
            lrow += FPB;
        }
        STAMP4(3);

        // ---- select (Horner in W_N^bin) + DDC + low-pass + phase, channels tid + 512 q ----
#pragma unroll
        for (int f = 0; f < FPB; ++f) {
            const int kf = kr + f;
            const float2* yf = fbuf + f * G::FB;
            float2 z[CPT];
#pragma unroll
            for (int q = 0; q < CPT; ++q) {
                // all eight reads of the channel issued before its Horner chain
                float2 yv[NW];
#pragma unroll
                for (int sg = 0; sg < NW; ++sg) yv[sg] = yf[yoff[q] + sg * G::REG];
                // two 4-term Horner chains joined by the exact W_N^{4 bin}: half the rounding
                // depth of one 8-term chain (the phase bar is 1e-5 rad), and two chains of ILP
                float2 Xl = yv[3], Xh = yv[7];
#pragma unroll
                for (int sg = 2; sg >= 0; --sg) {
                    Xl = cmac(yv[sg], Xl, tb[q]);
                    Xh = cmac(yv[sg + 4], Xh, tb[q]);
                }
                z[q] = cmul_pk(cmac(Xl, Xh, tb4[q]), lov[f][q]);
            }
            if ((f & 1) == 0) {
#pragma unroll
                for (int m = 0; m < 13; ++m)
#pragma unroll
                    for (int q = 0; q < CPT; ++q) acc[q][m] = fma_tap<1>(gp[m], z[q], acc[q][m]);   // g_{2m+1}
            } else {
                // output frame: accumulate and shift to the next output in one FMA each
                float2 y[CPT];
#pragma unroll
                for (int q = 0; q < CPT; ++q) y[q] = fma_tap<0>(gp[0], z[q], acc[q][0]);             // g_0
#pragma unroll
                for (int m = 0; m < 12; ++m)
#pragma unroll
                    for (int q = 0; q < CPT; ++q) acc[q][m] = fma_tap<0>(gp[m + 1], z[q], acc[q][m + 1]);  // g_{2m+2}
#pragma unroll
                for (int q = 0; q < CPT; ++q) acc[q][12] = make_float2(0.f, 0.f);
                if (kf > 0 && kf < nrun) {
                    const int jr = (kf - 1) >> 1;
                    float ph[CPT];
#pragma unroll
                    for (int q = 0; q < CPT; ++q) {
                        ys[q].x += y[q].x;
                        ys[q].y += y[q].y;
                        ph[q] = phase_atan2(y[q].y - qc[q], y[q].x - ic[q]);
                    }
#pragma unroll
                    for (int q = 0; q < CPT; ++q) {
                        const int c = tid + G::BT * q;
                        int qv = __float2int_rn(ph[q] * 8192.0f);
                        qv = qv < -25736 ? -25736 : (qv > 25736 ? 25736 : qv);
#ifndef MKID_XP_STAMPS
                        if (phase_run) __builtin_nontemporal_store(ph[q], phase_run + jr * C + c);
#endif
                        __builtin_nontemporal_store((int16_t)qv, raw_run + jr * C + c);
                        if (c == a.iq_ch && a.iqtap) {
                            a.iqtap[2 * ((k_b >> 1) + jr)] = iq16(y[q].x);
                            a.iqtap[2 * ((k_b >> 1) + jr) + 1] = iq16(y[q].y);
                        }
                    }
                }
            }
        }
        STAMP4(4);
        __syncthreads();  // select reads done before the next iteration's region writes
        STAMP4(5);
    }
    if (a.ysum)
#pragma unroll
        for (int q = 0; q < CPT; ++q) ysum_add(a.ysum, tid + G::BT * q, ys[q].x, ys[q].y);
}

bool front4_supported(int N) { return N == G4::N; }

hipError_t launch_front4(const FrontArgs& a0, hipStream_t s) {
    static std::atomic<uint64_t> attr_mask{0};
    hipError_t e = ensure_lds_attr(attr_mask, (const void*)k_front4, (int)G4::lds_bytes);
    if (e != hipSuccess) return e;
    FrontArgs a = a0;
    if (a.K <= 0) return hipSuccess;
    // runs of up to 1024 frames (the 24-frame low-pass warm-up is 2.3 % of a full run): a full
    // 2^30-sample chunk is two rounds of workgroups over the device's CUs (-2.2 % against 1024
    // runs of 512 frames on MI355X's 256 CUs, tools/kbench.py A/B)
    const int64_t ncu = a.ncu > 0 ? a.ncu : 256;
    int64_t fpb = a.K / (2 * ncu);
    fpb = fpb < 64 ? 64 : (fpb > 1024 ? 1024 : fpb);
    fpb = (fpb + G4::FPB - 1) / G4::FPB * G4::FPB;
    a.frames_per_block = fpb;
    const int64_t blocks = (a.K + fpb - 1) / fpb;
    hipLaunchKernelGGL(k_front4, dim3((unsigned)blocks), dim3(G4::BT), G4::lds_bytes, s, a);
    return hipGetLastError();
}

}  // namespace mkid
