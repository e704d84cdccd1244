// Fused front end v2 (N = 512, 1024, 2048): K1-K6 in one pass over the ADC stream, with an
// FFT that exchanges data between waves ONCE per frame and two workgroup barriers per iteration
// (v1, k_front.hip: three cross-wave LDS exchanges, six barriers).
//
// Decimation in time by NW = N/512: X[k] = sum_{w<NW} W_N^{w k} Y_w[k mod 512], where Y_w is the
// 512-point DFT of u[NW m + w]. Wave w of a frame computes Y_w entirely inside the wave:
//   lane L (0..63) holds v[r] = u[NW (64 r + L) + w], r = 0..7 (computed by the PFB straight from
//   the LDS ring), then
//   stage 1  radix-8 over r;            twiddle W_512^{L k}
//   T1       register bits <-> lane bits 3-5 through this wave's own LDS region (t1_lds; the
//            DPP / permlane-swap form cost more VALU issue than the LDS round trip)
//   stage 2  radix-8;                   twiddle W_64^{(L & 7) k}
//   T2       register bits <-> lane bits 0-2 through this wave's own LDS region (no barrier)
//   stage 3  radix-8 -> lane L, register r holds Y_w[(L >> 3) + 8 (L & 7) + 64 r]
//   write Y_w to the region (XOR-swizzled, conflict-free).
// Barrier. Thread c = channel c then evaluates only X[bin_c] = sum_w W_N^{w bin} Y_w[bin mod 512]
// (NW LDS reads, NW-1 complex MACs with per-channel constant twiddles) and runs the DDC,
// transposed decimating 26-tap low-pass, centre, atan2 and Fix16_13 exactly as k_front.hip.
// Barrier. Index maps checked by tools/front2_layouts.py (numpy emulation + bank-conflict check).
//
// LDS layouts (all conflict-free for their access patterns on gfx950):
//   ring   RS hops of M samples; sample offset o of a hop in plane (o % NW) (M / NW samples) at
//          plane index o / NW, paired (ring3_idx), so a lane's PFB points r, r + 1 of sub-FFT w are
//          one ds_read_b64
//   taps   the wave's PFB tap quads live in VGPRs (the same points every frame)
//   region per (frame, wave): 576 float2; T2 uses i + (i >> 3), Y uses k ^ ((k >> 2) & 14)
#include "front_common.h"

#ifdef MKID_XP_STAMPS
#define FSYNC2(id)                 \
    do {                           \
        STAMP2(2 * (id));          \
        __syncthreads();           \
        STAMP2(2 * (id) + 1);      \
    } while (0)
#define STAMP2(slot_)                                                                             \
    do {                                                                                          \
        __builtin_amdgcn_sched_barrier(0);                                                        \
        const uint64_t tm_ = __builtin_amdgcn_s_memtime();                                        \
        __builtin_amdgcn_sched_barrier(0);                                                        \
        if (blockIdx.x < 4 && it_ >= 8 && it_ < 16 && (threadIdx.x & 63) == 0)                   \
            reinterpret_cast<uint64_t*>(a.phase)[((blockIdx.x * 16 + (threadIdx.x >> 6)) * 8 +   \
                                                  (it_ - 8)) * 16 + (slot_)] = tm_;               \
    } while (0)
#else
#define FSYNC2(id) __syncthreads()
#define STAMP2(slot_) ((void)0)
#endif

namespace mkid {

namespace {

template <int N>
struct G2 {
    static constexpr int NW = N / 512;                 // waves (512-point sub-FFTs) per frame
    static constexpr int FPB = 4;                      // frames per iteration
    static constexpr int BT = FPB * NW * 64;           // threads == channels
    static constexpr int M = N / 2, C = N / 2, T = kPfbTaps;
    static constexpr int RS = 2 * T - 1 + FPB;         // ring slots (hops)
    static constexpr int REG = 576;                    // float2 per (frame, wave) region
    static constexpr int FB = NW * REG;                // float2 per frame
    static constexpr size_t off_fbuf = (size_t)RS * M * 4;
    static constexpr size_t off_tw1 = off_fbuf + (size_t)FPB * FB * 8;  // W_512^{L k}: [k-1][L]
    static constexpr size_t off_tw2 = off_tw1 + (size_t)7 * 64 * 8;    // W_64^{l k}: [k-1][l]
    static constexpr size_t lds_bytes = off_tw2 + (size_t)7 * 8 * 8;
    static_assert(BT == C, "one channel per thread");
    static_assert(N >= 512 && N <= 2048, "v2 geometry");
};

// Ring planes in the paired layout (every plane is Q = M / NW = 256 samples): samples qoff..qoff+3
// of a hop go to plane (o mod NW), plane index o / NW, at ring3_idx of it (qoff is a multiple of 4,
// so the 4 indices of a plane stay in one 64-block and ring3_idx steps by 2). The refill's
// ds_write_b32 become 2-way bank conflicts, free for 4-byte stores (MI355X_MICROARCH.md §LDS).
template <int N>
__device__ __forceinline__ void ring_put_paired(uint32_t* hop, int qoff, uint4 v) {
    using G = G2<N>;
    constexpr int Q = G::M / G::NW;
    static_assert(Q == 256, "paired plane layout");
    if constexpr (G::NW == 1) {
        const int a = ring3_idx(qoff);
        hop[a] = v.x;
        hop[a + 2] = v.y;
        hop[a + 4] = v.z;
        hop[a + 6] = v.w;
    } else if constexpr (G::NW == 2) {
        const int a = ring3_idx(qoff / 2);
        hop[a] = v.x;
        hop[a + 2] = v.z;
        hop[Q + a] = v.y;
        hop[Q + a + 2] = v.w;
    } else {
        const int a = ring3_idx(qoff / 4);
        hop[a] = v.x;
        hop[Q + a] = v.y;
        hop[2 * Q + a] = v.z;
        hop[3 * Q + a] = v.w;
    }
}

}  // namespace


template <int N>
__global__ __launch_bounds__(G2<N>::BT, 4) void k_front2(FrontArgs a) {
    using G = G2<N>;
    constexpr int NW = G::NW, M = G::M, C = G::C, T = G::T, RS = G::RS, FPB = G::FPB;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t* ring = reinterpret_cast<uint32_t*>(smem);
    float2* fbuf = reinterpret_cast<float2*>(smem + G::off_fbuf);
    float2* tw1 = reinterpret_cast<float2*>(smem + G::off_tw1);
    float2* tw2 = reinterpret_cast<float2*>(smem + G::off_tw2);

    const int tid = threadIdx.x;
    const int L = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int slot = wave / NW;   // frame of the iteration this wave transforms
    const int w = wave % NW;      // its sub-FFT
    float2* reg = fbuf + slot * G::FB + w * G::REG;

    // stage-1/2 twiddle tables
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

    // select stage constants of channel c = tid: X[bin] = sum_w W_N^{w bin} Y_w[bin mod 512]
    const int c = tid;
    const int32_t bin = a.bins[c];
    const float ic = a.ic[c], qc = a.qc[c];
    float2 tl[NW > 1 ? NW - 1 : 1];
#pragma unroll
    for (int q = 1; q < NW; ++q) {
        double sn, cs;
        sincospi(-2.0 * (double)((q * bin) % N) / N, &sn, &cs);
        tl[q - 1] = make_float2((float)cs, (float)sn);
    }
    const int yoff = yswz(bin & 511);
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
    [[maybe_unused]] float* const phase_run = a.phase ? a.phase + (k_b >> 1) * C : nullptr;

    const int qh = (tid * 4) / M, qoff = (tid * 4) % M;  // this thread's ring write
    // prologue: hops k_start-2T+1 .. k_start+FPB-1 -> ring (slot = hop mod RS)
    {
        const int64_t h0 = k_start - 2 * T + 1;
        for (int g = 0; g < RS; g += FPB) {
            const int64_t hop = h0 + g + qh;
            if (hop > h0 + RS - 1) continue;
            const uint4 v = front_load4<M>(a, h0 + g, tid);
            ring_put_paired<N>(ring + (int)(((hop % RS) + RS) % RS) * M, qoff, v);
        }
    }
    __syncthreads();

    float2 acc[13];
#pragma unroll
    for (int m = 0; m < 13; ++m) acc[m] = make_float2(0.f, 0.f);
    float2 ys = make_float2(0.f, 0.f);

    int rb = (int)((((k_start + 1 - 2 * T) % RS) + RS) % RS);
    int lrow = (int)((a.k0 + k_start) & (int64_t)(a.P - 1));
    const int nrun = (int)(k_e - k_b);
    // per-lane LDS bases of the in-wave exchange and the Y write (all offsets below immediates)
    const int la = L & 7, kl = L >> 3;
    float2* t2w = reg + 72 * kl + la;        // T2 write: i = 64 kl + 8 r + la  -> i + (i >> 3)
    const float2* t2r = reg + 72 * kl + 9 * la;  // T2 read: i = 64 kl + 8 la + r
    float2* yw = reg + ((kl + 8 * la) ^ (la << 1));   // Y: k = kl + 8 la + 64 r, swizzled
    // the wave's points are the same every frame: tap quads in VGPRs instead of LDS reads
    uint2 tq[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) tq[r] = a.pfbq[NW * (64 * r + L) + w];
    const float2* t1 = tw1 + L;               // W_512^{L k} at t1[64 (k - 1)]
    const float2* t2 = tw2 + la;              // W_64^{la k} at t2[8 (k - 1)]

#ifdef MKID_XP_STAMPS
    int it_ = 0;
#endif
    for (int kr = -kLpfHist; kr < nrun; kr += FPB) {
#ifdef MKID_XP_STAMPS
        ++it_;
        STAMP2(14);
#endif
        // this iteration's ring refill (written after the FFT barrier), loaded first: no ring
        // load is outstanding in the select phase (vmcnt waits are in issue order)
        const uint4 pre = front_load4<M>(a, k_b + kr + FPB, tid);
        float2 lov[FPB];
#pragma unroll
        for (int f = 0; f < FPB; ++f) lov[f] = (a.lo + ((lrow + f) & (a.P - 1)) * C)[c];

        // ---- PFB: points NW (64 r + L) + w of frame kb + slot ----
        int sb = rb + slot;
        sb -= sb >= RS ? RS : 0;
        float2 v[8];
        uint32_t xo[T];   // the odd point's samples (paired planes)
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const int hi = r >> 2;
            const uint64_t h64 = (uint64_t)tq[r].x | ((uint64_t)tq[r].y << 32);
            uint32_t x4[T];
            // points r, r + 1 (r even) are one ds_read_b64 of the paired plane layout: read at the
            // even point, kept for the odd one
            static_assert(T == 4, "taps");
            if ((r & 1) == 0) {
#pragma unroll
                for (int tau = 0; tau < T; ++tau) {
                    int sl = sb + 2 * tau + hi;
                    sl -= sl >= RS ? RS : 0;
                    const uint2 p = *reinterpret_cast<const uint2*>(ring + sl * M + w * (M / NW) + 128 * ((r & 3) >> 1) + 2 * L);
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
            int32_t ai = dot2_first((uint32_t)h64, i01);
            ai = __builtin_amdgcn_sdot2(as_s2((uint32_t)(h64 >> 32)), as_s2(i23), ai, false);
            int32_t aq = dot2_first((uint32_t)h64, q01);
            aq = __builtin_amdgcn_sdot2(as_s2((uint32_t)(h64 >> 32)), as_s2(q23), aq, false);
            v[r] = make_float2((float)ai, (float)aq);
            if ((r & 3) == 3)
                asm volatile("" : "+v"(v[r].x), "+v"(v[r].y), "+v"(v[r - 1].x), "+v"(v[r - 1].y),
                             "+v"(v[r - 2].x), "+v"(v[r - 2].y), "+v"(v[r - 3].x), "+v"(v[r - 3].y));
        }
        // ---- stage 1 + twiddle W_512^{L k} ----
        dft<8>(v);
#pragma unroll
        for (int k = 1; k < 8; ++k) v[k] = cmul_pk(v[k], t1[64 * (k - 1)]);
        // ---- T1 through the wave's own LDS region + stage 2 + twiddle ----
        t1_lds(v, reg, L);
        dft<8>(v);
#pragma unroll
        for (int k = 1; k < 8; ++k) v[k] = cmul_pk(v[k], t2[8 * (k - 1)]);
        // ---- T2 through the wave's own region (no workgroup barrier) ----
#pragma unroll
        for (int r = 0; r < 8; ++r) t2w[9 * r] = v[r];
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int r = 0; r < 8; ++r) v[r] = t2r[r];
        dft<8>(v);
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int r = 0; r < 8; ++r) yw[64 * r] = v[r];
        FSYNC2(0);  // Y of all frames visible; every ring read of this iteration done

        {   // ring refill for the next iteration (its oldest FPB hops), prefetch one further
            int ws = rb + qh;
            ws -= ws >= RS ? RS : 0;
            ring_put_paired<N>(ring + ws * M, qoff, pre);
            rb += FPB;
            rb -= rb >= RS ? RS : 0;
            lrow += FPB;
        }

        // ---- select + DDC + low-pass + phase for channel c over the FPB frames ----
#pragma unroll
        for (int f = 0; f < FPB; ++f) {
            const int kf = kr + f;
            const float2* yf = fbuf + f * G::FB + yoff;
            float2 X = yf[0];
#pragma unroll
            for (int q = 1; q < NW; ++q) X = cmac(X, tl[q - 1], yf[q * G::REG]);
            const float2 z = cmul_pk(X, lov[f]);
            if ((f & 1) == 0) {
#pragma unroll
                for (int m = 0; m < 13; ++m) acc[m] = fma_tap<1>(gp[m], z, acc[m]);   // g_{2m+1}
            } else {
                // output frame: the accumulate and the shift to the next output are one FMA per
                // accumulator (acc[m] <- acc[m+1] + g_{2m+2} z), no register moves
                const float2 y = fma_tap<0>(gp[0], z, acc[0]);                          // g_0
#pragma unroll
                for (int m = 0; m < 12; ++m) acc[m] = fma_tap<0>(gp[m + 1], z, acc[m + 1]);  // g_{2m+2}
                acc[12] = make_float2(0.f, 0.f);
                if (kf > 0 && kf < nrun) {
                    const int jr = (kf - 1) >> 1;
                    ys.x += y.x;
                    ys.y += y.y;
                    const float ph = phase_atan2(y.y - qc, y.x - ic);
                    int q = __float2int_rn(ph * 8192.0f);
                    q = q < -25736 ? -25736 : (q > 25736 ? 25736 : q);
#ifndef MKID_XP_STAMPS
                    if (phase_run) __builtin_nontemporal_store(ph, phase_run + jr * C + c);
#endif
                    __builtin_nontemporal_store((int16_t)q, raw_run + jr * C + c);
                    if (c == a.iq_ch && a.iqtap) {
                        a.iqtap[2 * ((k_b >> 1) + jr)] = iq16(y.x);
                        a.iqtap[2 * ((k_b >> 1) + jr) + 1] = iq16(y.y);
                    }
                }
            }
        }
        FSYNC2(1);  // select reads done before the next iteration's region writes
    }
    if (a.ysum) ysum_add(a.ysum, c, ys.x, ys.y);
}

bool front2_supported(int N) { return N == 512 || N == 1024 || N == 2048; }

template <int N>
static hipError_t launch_front2_n(const FrontArgs& a0, hipStream_t s) {
    using G = G2<N>;
    static std::atomic<uint64_t> attr_mask{0};
    hipError_t e = ensure_lds_attr(attr_mask, (const void*)k_front2<N>, (int)G::lds_bytes);
    if (e != hipSuccess) return e;
    FrontArgs a = a0;
    if (a.K <= 0) return hipSuccess;
    // one round of workgroups over the device's CUs for a large chunk (2048/N workgroups fit a CU:
    // the LDS plan scales with N), runs of <= 4096 frames: at N = 2048 a 2^30-sample chunk is one
    // 4096-frame run per CU of MI355X's 256, the 24-frame low-pass warm-up 0.6 % of it (-1.4 %
    // against 1024 runs of 1024 frames, tools/kbench.py A/B)
    const int64_t ncu = a.ncu > 0 ? a.ncu : 256;
    int64_t fpb = a.K / (ncu * (2048 / N));
    fpb = fpb < 64 ? 64 : (fpb > 4096 ? 4096 : fpb);
    fpb = (fpb + G::FPB - 1) / G::FPB * G::FPB;
    a.frames_per_block = fpb;
    const int64_t blocks = (a.K + fpb - 1) / fpb;
    hipLaunchKernelGGL(k_front2<N>, dim3((unsigned)blocks), dim3(G::BT), G::lds_bytes, s, a);
    return hipGetLastError();
}

hipError_t launch_front2(int N, const FrontArgs& a, hipStream_t s) {
    if ((N == 2048 || N == 512) && a.variant == 3) return launch_front3(N, a, s);
    switch (N) {
        case 512: return launch_front2_n<512>(a, s);
        case 1024: return launch_front2_n<1024>(a, s);
        case 2048: return launch_front2_n<2048>(a, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace mkid
