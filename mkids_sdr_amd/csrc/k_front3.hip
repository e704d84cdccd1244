// Fused front end k_front3 (N = 2048, config 3/4; the default at N = 2048): k_front2's arithmetic
// (k_front2.hip) with wave specialisation.
#include "front_common.h"

namespace mkid {

namespace {
// Pair ring (round 4). The PFB of point p, frame k is sum_tau h_tau x[hop k - 7 + hi + 2 tau][o]
// (hi = p / M, o = p mod M), evaluated as two v_dot2_i32_i16 per component over 16-bit pairs
// (x[s], x[s + 2]) of the same offset two hops apart. Those pairs used to be built per point per
// frame with 4 v_perm from the interleaved I/Q words; every sample is read by 8 (frame, point)
// PFB evaluations, so the ring now stores the pairs themselves, built once at refill: pair-hop
// P(s)[o] = (I pair, Q pair) = ({I x[s][o], I x[s+2][o]}, {Q x[s][o], Q x[s+2][o]}), 8 bytes.
// The refill thread that loads hop s + 2 at offsets o..o+3 loaded hop s at the same offsets one
// iteration earlier and kept it in registers (`prev`), so a pair costs one v_perm per component
// (2 per sample, against 8 per sample before).
// Layout of a pair-hop (1024 samples, 8 KiB): plane u = o % 4 (256 entries of 8 B), plane index
// i = o / 4 at entry ring3_idx(i), so a lane's points j, j + 1 (i = 64 j + L, j even) are one
// conflict-free ds_read_b128. Refill thread g' (0..255 of its hop) owns plane index
// i = 128 (g' >> 7) + ((g' >> 1) & 63) + 64 (g' & 1), whose entry is ring3_idx(i) = g': each of its
// four ds_write_b64 (one per plane) is consecutive across lanes, conflict-free.
__device__ __forceinline__ int pair_owner_index(int g) { return 128 * (g >> 7) + ((g >> 1) & 63) + 64 * (g & 1); }
__device__ __forceinline__ void pair_put(uint2* phop, int g, uint4 prev, uint4 cur) {
    phop[g] = make_uint2(__builtin_amdgcn_perm(cur.x, prev.x, kPermI), __builtin_amdgcn_perm(cur.x, prev.x, kPermQ));
    phop[256 + g] = make_uint2(__builtin_amdgcn_perm(cur.y, prev.y, kPermI), __builtin_amdgcn_perm(cur.y, prev.y, kPermQ));
    phop[512 + g] = make_uint2(__builtin_amdgcn_perm(cur.z, prev.z, kPermI), __builtin_amdgcn_perm(cur.z, prev.z, kPermQ));
    phop[768 + g] = make_uint2(__builtin_amdgcn_perm(cur.w, prev.w, kPermI), __builtin_amdgcn_perm(cur.w, prev.w, kPermQ));
}
}  // namespace
// In k_front2 every wave runs the FFT phase, then every wave runs the select phase, with a
// workgroup barrier between them: when all four waves of a SIMD wait on LDS (ring reads, the
// select's bin-indexed reads) or on a barrier, the SIMD idles (stamps: the FFT phase of the last
// wave of a SIMD ends ~2.4k cycles after the first, VALU busy ~70 %). Here waves 0-7 only transform
// (2 frames per iteration, one 512-point sub-FFT each) and waves 8-15 only select / mix / low-pass /
// phase (two channels per thread), one iteration behind, on a double-buffered Y: each SIMD holds
// two FFT and two select waves whose LDS waits and VALU bursts interleave, one barrier per
// iteration.
//   ring  RS = 9 pair-hops P(s) (above): iteration t (frames k, k+1) reads P(k-7) .. P(k-1) while
//         its FFT waves write P(k), P(k+1) (from hops k+2, k+3, prefetched at the loop top, and the
//         hops k, k+1 each refill thread kept) over P(k-9), P(k-8)
//   Y     [2][F][NW][576] float2, iteration t writes buffer t & 1, its select reads (t - 1) & 1
// Registers: the FFT path holds the PFB taps and the 512-point sub-FFT, the select path two
// channels' low-pass state; branches are wave-uniform, so the two live sets do not add up.
// Measured and dropped: LDS progress words instead of the barrier on three Y
// buffers (+5.6 %), roles alternating by age on each SIMD (+2.6 %), issue priority for either
// group or for the younger wave of a pair (zero-sum), non-temporal raw / phase stores (+1.3 %).

template <int N>
struct G3 {
    static constexpr int NW = N / 512;
    static constexpr int FW = 8;                       // transform waves
    static constexpr int F = FW / NW;                  // frames per iteration
    static constexpr int BT = 1024;
    static constexpr int SPT = BT - FW * 64;           // select threads
    static constexpr int M = N / 2, C = N / 2, T = kPfbTaps;
    static constexpr int CPT = C / SPT;                // channels per select thread
    static constexpr int RS = 2 * T - 1 + F;           // ring slots (pair-hops of M x 8 B)
    static constexpr int REG = 576;
    static constexpr int FB = NW * REG;
    static constexpr size_t off_fbuf = (size_t)RS * M * 8;
    static constexpr int NB = 2;                       // Y buffers
    static constexpr size_t off_tw1 = off_fbuf + (size_t)NB * F * FB * 8;
    static constexpr size_t off_tw2 = off_tw1 + (size_t)7 * 64 * 8;
    static constexpr size_t lds_bytes = off_tw2 + (size_t)7 * 8 * 8;
    static_assert(N == 2048 && F == 2 && CPT == 2 && F * M == FW * 64 * 4 && T == 4, "k_front3 geometry");
    static_assert(lds_bytes <= 160 * 1024, "LDS");
};

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
__global__ __launch_bounds__(G3<N>::BT, 4) void k_front3(FrontArgs a) {
    using G = G3<N>;
    constexpr int NW = G::NW, M = G::M, C = G::C, RS = G::RS, F = G::F, CPT = G::CPT;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint2* ring = reinterpret_cast<uint2*>(smem);
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
        // refill: waves 0-3 (qh = 0) own the even hop of each pair of new hops, waves 4-7 the odd
        // one; thread g' of its hop loads samples 4 i .. 4 i + 3, i = pair_owner_index(g')
        const int qh = rw >> 2, gp = (rw & 3) * 64 + L;
        const int xl = qh * (M / 4) + pair_owner_index(gp);   // front_load4 index: sample 4 xl of the 2 hops
        uint4 prev = make_uint4(0, 0, 0, 0);                   // hop h - 2 at the same offsets
        {   // prologue: hops k_start - 7 .. k_start + 1 -> P(k_start - 7) .. P(k_start - 1); hop
            // k_start - 8 (qh = 0, m = 0) is neither needed nor inside the history
#pragma unroll
            for (int m = 0; m <= 4; ++m) {
                if (qh == 0 && m == 0) continue;
                const uint4 cur = front_load4<M>(a, k_start - 8 + 2 * m, xl);
                const int64_t s_ = k_start - 10 + 2 * m + qh;   // pair-hop of (h - 2, h)
                if (m > 0 && s_ >= k_start - 7) pair_put(ring + (int)(((s_ % RS) + RS) % RS) * M, gp, prev, cur);
                prev = cur;
            }
        }
        uint2 tq[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) tq[r] = a.pfbq[NW * (64 * r + L) + w];
        const int la = L & 7, kl = L >> 3;
        const float2* t1 = tw1 + L;
        const float2* t2 = tw2 + la;
        int rb = (int)((((k_start - 7) % RS) + RS) % RS);   // slot of P(k - 7)
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
        for (int t = 0; t <= nit; ++t) {
            STAMP3(0);
            if (t < nit) {
                const int kr = -kLpfHist + F * t;
                // the hops iteration t + 1 adds: loaded now, written after this wave's PFB
                const uint4 pre = front_load4<M>(a, k_b + kr + F, xl);
                float2* reg = fbuf + ((t % G::NB) * F + slot) * G::FB + w * G::REG;
                int sb = rb + slot;
                sb -= sb >= RS ? RS : 0;
                // pair words of points 4 hi + 2 jp + {0, 1} from P(s) (taps 0, 1) and P(s + 4)
                // (taps 2, 3), s = k + slot - 7 + hi: 8 ds_read_b128
                uint4 pw[2][2][2];
#pragma unroll
                for (int hi = 0; hi < 2; ++hi)
#pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        int sl = sb + hi + 4 * e;
                        sl -= sl >= RS ? RS : 0;
                        const uint4* pl = reinterpret_cast<const uint4*>(ring + sl * M + w * (M / NW)) + L;
                        pw[hi][0][e] = pl[0];
                        pw[hi][1][e] = pl[64];
                    }
                float2 v[8];
#pragma unroll
                for (int r = 0; r < 8; ++r) {
                    const uint4& p0 = pw[r >> 2][(r >> 1) & 1][0];
                    const uint4& p1 = pw[r >> 2][(r >> 1) & 1][1];
                    const uint32_t i01 = (r & 1) ? p0.z : p0.x, q01 = (r & 1) ? p0.w : p0.y;
                    const uint32_t i23 = (r & 1) ? p1.z : p1.x, q23 = (r & 1) ? p1.w : p1.y;
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
                // ring refill: P(k + qh) = (hop k + qh, hop k + 2 + qh) into the slot of P(k - 9 + qh)
                // (no reader this iteration)
                int ws = rb + 7 + qh;
                ws -= ws >= RS ? RS : 0;
                pair_put(ring + ws * M, gp, prev, pre);
                prev = pre;
                rb += F;
                rb -= rb >= RS ? RS : 0;
            }
            STAMP3(1);
            __syncthreads();
            STAMP3(2);
        }
    } else {
        // ---------------- select waves: channels st + SPT q, one iteration behind ---------------
        const int st = rw * 64 + L;
        float2 tl[CPT][NW - 1];
        int yoff[CPT];
        float ic[CPT], qc[CPT];
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
            ic[q] = a.ic[c];
            qc[q] = a.qc[c];
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
        // the run's outputs (<= 2048 rows x C) and the LO table (P x C float2 = 512 KiB) through
        // buffer descriptors: row offsets in SGPRs, the lanes' channel offsets loop-invariant
        const __amdgpu_buffer_rsrc_t raw_rs = buf_rsrc(raw_run);
        const __amdgpu_buffer_rsrc_t ph_rs = buf_rsrc(phase_run ? phase_run : a.phase);
        const __amdgpu_buffer_rsrc_t lo_rs = buf_rsrc(a.lo);
        int lrow = (int)((a.k0 + k_start) & (int64_t)(a.P - 1));
        __syncthreads();
        for (int t = 0; t <= nit; ++t) {
            STAMP3(3);
            if (t > 0) {
                const int kr = -kLpfHist + F * (t - 1);
                float2 lov[F][CPT];
#pragma unroll
                for (int f = 0; f < F; ++f) {
                    const uint32_t row = (uint32_t)(((lrow + f) & (a.P - 1)) * C) * 8u;
#pragma unroll
                    for (int q = 0; q < CPT; ++q) lov[f][q] = buf_ld_f2(lo_rs, 8u * (uint32_t)cq[q], row);
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
                        z[q] = cmul_pk(X, lov[f][q]);
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
                                const float ph = phase_atan2(y[q].y - qc[q], y[q].x - ic[q]);
                                int qv = __float2int_rn(ph * 8192.0f);
                                qv = qv < -25736 ? -25736 : (qv > 25736 ? 25736 : qv);
                                // plain stores: with the slot order a wave's store covers its 64
                                // channels within 2 (raw) or 4 (phase) lines, merged in L2
#ifndef MKID_XP_STAMPS   // the timing build keeps its stamps in the phase buffer
                                if (phase_run) buf_st_f32(ph_rs, 4u * (uint32_t)c, 4u * (uint32_t)(jr * C), ph);
#endif
                                buf_st_i16(raw_rs, 2u * (uint32_t)c, 2u * (uint32_t)(jr * C), (int16_t)qv);
                                if (c == a.iq_ch && a.iqtap) {
                                    a.iqtap[2 * ((k_b >> 1) + jr)] = iq16(y[q].x);
                                    a.iqtap[2 * ((k_b >> 1) + jr) + 1] = iq16(y[q].y);
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
    int64_t fpb = a.K / ncu;                     // one run per CU, as k_front2
    fpb = fpb < 64 ? 64 : (fpb > 4096 ? 4096 : fpb);
    fpb = (fpb + G::F - 1) / G::F * G::F;
    a.frames_per_block = fpb;
    const int64_t blocks = (a.K + fpb - 1) / fpb;
    hipLaunchKernelGGL(k_front3<N>, dim3((unsigned)blocks), dim3(G::BT), G::lds_bytes, s, a);
    return hipGetLastError();
}

hipError_t launch_front3(const FrontArgs& a, hipStream_t s) { return launch_front3_n<2048>(a, s); }

}  // namespace mkid
