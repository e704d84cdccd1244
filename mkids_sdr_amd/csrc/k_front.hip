// Fused front end for N = 128 / 256 (configs[0]'s 64-channel geometry; N >= 512 runs the
// wave-specialised k_front3 / k_front5, launch_fused below).
// K1-K6 in one pass over the ADC stream: polyphase filter bank + N-point FFT
// (2x oversampled, hop M = N/2) + bin select + DDC + 26-tap IQ low-pass decimating by 2 +
// IQ-centre subtraction + atan2 + Fix16_13. The complex baseband z never leaves the CU: HBM sees
// 4 B/sample of int16 I/Q in and 1 B/sample of raw phase (+2 B/sample float phase) out.
//
// A workgroup of BT = N/2 = C threads owns a contiguous run of frames [k_b, k_e) and walks it
// FPB = 4 frames per iteration (NT = N/8 threads per frame, 8 points per thread):
//   input  LDS ring of RS = 2T-1+FPB hops of M int16 I/Q samples; each iteration brings 4 new
//          hops with ONE 16-byte global load per thread, issued one iteration ahead.
//   PFB    u[p] = sum_tau h_q[tau N + p] x[(k+1)M - TN + tau N + p]: exact int16 dot products
//          (taps h_q = rint(h 2^S), mkid_set_pfb; the 2^-S rides in the LO table)
//   FFT    Stockham radix-8/4 passes through a padded per-frame LDS buffer (fft_common.h); the
//          last pass is fused into the select: thread c evaluates only the radix-4 butterfly
//          output X[bin_c] (4 LDS reads, 3 complex MACs with per-channel constant twiddles).
//   DDC    thread c = channel c: z_k = X_k[bin_c] (-1)^(bin_c (k+1)) conj(LUT_c[k mod P]) / 2^15
//          for the 4 frames of the iteration (LO table [P][C]: one contiguous row per frame; the
//          bin-parity sign is folded into the table on the host, P being even).
//   LPF    transposed form, 13 complex accumulators per thread: frame 2j adds g_{2m+1} z to
//          output j+m, frame 2j+1 adds g_{2m} z and completes output j:
//          y_j = sum_i g_i z_{2j+1-i}      (taps int(lpf*(2**11-1))/2^11, ROACH_Pulses.py:69,88)
//   phase  phi_j = atan2(Im y - qc, Re y - ic)     (pulse_triggering_IQ.py:152), accumulated
//          centred: y - c = sum_i g_i (z_i - c') + r  (mkid_internal.h Centring)
//          raw_j = clamp(rint(phi_j 2^13), +-25736) (Fix16_13, ROACH_Pulses.py:274-278)
// Each run starts kLpfHist = 24 frames early (warm-up: the low-pass history is recomputed from
// the ADC samples instead of being stored), so frames before the chunk come from an ADC history
// of (2T-1+24) hops carried between calls. Reference geometry: ROACH_Setup.py:507-550.
#include "fft_common.h"
#include "mkid_internal.h"

// MKID_XP_STAMPS (timing experiments only, tools/stamps.py): lane 0 of every wave of the first
// 4 workgroups records s_memtime before and after each barrier of iterations 8..15 into the
// phase buffer (which then holds no phases).
#ifdef MKID_XP_STAMPS
#define FSYNC(id)                  \
    do {                           \
        STAMP(2 * (id));           \
        __syncthreads();           \
        STAMP(2 * (id) + 1);       \
    } while (0)
#define STAMP(slot_)                                                                              \
    do {                                                                                          \
        __builtin_amdgcn_sched_barrier(0);                                                        \
        const uint64_t tm_ = __builtin_amdgcn_s_memtime();                                        \
        __builtin_amdgcn_sched_barrier(0);                                                        \
        if (blockIdx.x < 4 && it_ >= 8 && it_ < 16 && (threadIdx.x & 63) == 0)                   \
            reinterpret_cast<uint64_t*>(a.phase)[((blockIdx.x * 16 + (threadIdx.x >> 6)) * 8 +   \
                                                  (it_ - 8)) * 16 + (slot_)] = tm_;               \
    } while (0)
#else
#define FSYNC(id) __syncthreads()
#define STAMP(slot_) ((void)0)
#endif

// Streaming traffic is non-temporal: the ADC stream is read once and the phase rows are written
// once, so neither should evict the LO table (512 KB at 1024 channels, re-read by every
// workgroup every iteration) from L2. With default-policy streams the LO rows miss L2 on some
// boxes and their loads stall the select stage: same-box A/B -15 % k_front, -11 % k_trigger
// (profiles/r01/r01_v29_kbench_nt.json). 0 restores default-policy accesses for A/B.

namespace mkid {

typedef short fshort2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ fshort2_t as_s2(uint32_t v) { return __builtin_bit_cast(fshort2_t, v); }
// First dot product of a chain: the VOP3P form with an inline-constant zero accumulator (the
// compiler otherwise picks v_dot2c_i32_i16 behind a v_mov of 0)
__device__ __forceinline__ int32_t dot2_i16_first(uint32_t h, uint32_t x) {
    int32_t d;
    asm("v_dot2_i32_i16 %0, %1, %2, 0" : "=v"(d) : "v"(h), "v"(x));
    return d;
}

// Radix sequence per FFT length (8 points per thread). The last pass is not run through LDS:
// its radix-RL butterfly is evaluated only for the selected bin, by the channel's thread.
template <int N>
struct FPlan;
template <> struct FPlan<128>  { static constexpr int NP = 3, R[4] = {8, 4, 4, 1}; };
template <> struct FPlan<256>  { static constexpr int NP = 3, R[4] = {8, 8, 4, 1}; };
template <> struct FPlan<512>  { static constexpr int NP = 4, R[4] = {8, 4, 4, 4}; };
template <> struct FPlan<1024> { static constexpr int NP = 4, R[4] = {8, 8, 4, 4}; };
template <> struct FPlan<2048> { static constexpr int NP = 4, R[4] = {8, 8, 8, 4}; };

template <int N>
struct FGeo {
    static constexpr int PTS = 8, NT = N / PTS, FPB = 4;
    static constexpr int BT = NT * FPB;                 // == C: one channel per thread
    static constexpr int M = N / 2, C = N / 2, T = kPfbTaps;
    static constexpr int RS = 2 * T - 1 + FPB;          // ring slots (hops)
    // exchange B (pass-2 write -> pass-3 read; plans with 4 passes) layout: conflict-free at
    // N >= 1024, half the read cycles of Pad16 at N = 512 (tools/lds_layouts.py)
    using PadB = LPad<5, 4>;
    static constexpr int LDSF = (Pad16::size(N) > PadB::size(N) ? Pad16::size(N) : PadB::size(N)) + 1 & ~1;
    static constexpr int SPT = FPB * M / BT;            // new samples per thread per iteration
    static_assert(SPT == 4, "one 16-byte load per thread per iteration");
    static_assert(BT == C, "one channel per thread");
    static constexpr int NS2 = FPlan<N>::R[0], NS3 = NS2 * FPlan<N>::R[1];
    static constexpr int RL = FPlan<N>::R[FPlan<N>::NP - 1];  // radix of the fused last pass
    static constexpr int NSL = N / RL;                        // its butterfly count / stride
    static_assert(NSL % 16 == 0, "pad-linear offsets in the fused last pass");
    using TW2 = TwiddleLds<N, PTS, FPlan<N>::R[1], NS2>;
    using TW3 = TwiddleLds<N, PTS, (FPlan<N>::NP == 4 ? FPlan<N>::R[2] : 2), NS3>;
    static constexpr size_t tw_offset = (size_t)RS * M * 4 + (size_t)FPB * LDSF * 8 + (size_t)N * 8;
    static constexpr size_t lds_bytes = tw_offset + (size_t)(TW2::ENTRIES + TW3::ENTRIES) * 8;
    static constexpr int HIST = (2 * T - 1 + kLpfHist) * M;  // ADC history samples
    // register budget sized for 4 waves per SIMD (16 per CU, <= 128 VGPRs): HIP's second
    // launch-bounds argument is the minimum waves per execution unit
    static constexpr int MINW = 4;
};

// The 16 bytes (4 samples) this thread contributes to the FPB hops starting at first_hop.
template <int N>
__device__ __forceinline__ uint4 front_load(const FrontArgs& a, int64_t first_hop, int tid) {
    using G = FGeo<N>;
    const int64_t s0 = first_hop * G::M + (int64_t)tid * G::SPT;  // sample index in chunk
    if (s0 >= a.K * G::M) return make_uint4(0, 0, 0, 0);
    if (s0 >= -a.avail) {
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a.x + s0));
        return make_uint4(v.x, v.y, v.z, v.w);
    }
    return *reinterpret_cast<const uint4*>(a.xhist + (s0 + a.avail + G::HIST));
}

template <int N>
__global__ __launch_bounds__(FGeo<N>::BT, FGeo<N>::MINW) void k_front(FrontArgs a) {
    using G = FGeo<N>;
    using PL = FPlan<N>;
    constexpr int PTS = G::PTS, NT = G::NT, M = G::M, C = G::C, T = G::T, RS = G::RS, FPB = G::FPB;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t* ring = reinterpret_cast<uint32_t*>(smem);
    float2* fbuf = reinterpret_cast<float2*>(smem + (size_t)RS * M * 4);

    const int tid = threadIdx.x;
    // frame of the iteration this thread transforms: wave-uniform when a wave lies within one
    // frame (NT >= 64), so the ring-slot arithmetic below runs on the scalar unit
    const int slot = NT % 64 == 0 ? __builtin_amdgcn_readfirstlane(tid / NT) : tid / NT;
    const int t = tid % NT;
    float2* buf = fbuf + slot * G::LDSF;
    // PFB taps of point p as int16 pairs {h0|h1, h2|h3} in LDS (8 B per point): the PFB is an
    // exact int16 x int16 dot product per I/Q component (v_dot2_i32_i16), the tap scale 2^-S
    // rides in the LO table
    uint2* hl = reinterpret_cast<uint2*>(smem + (size_t)RS * M * 4 + (size_t)FPB * G::LDSF * 8);
    static_assert(T == 4, "two int16 tap pairs per point");
    for (int p = tid; p < N; p += G::BT) hl[p] = a.pfbq[p];

    // pass-2/3 twiddle tables in LDS (filled once; published by the prologue barrier)
    float2* twt = reinterpret_cast<float2*>(smem + G::tw_offset);
    typename G::TW2 tw2{twt};
    typename G::TW3 tw3{twt + G::TW2::ENTRIES};
    G::TW2::fill(twt, tid, G::BT);
    if constexpr (PL::NP == 4) G::TW3::fill(twt + G::TW2::ENTRIES, tid, G::BT);

    const int c = tid;  // channel of the select / low-pass / phase stage
    const int32_t bin = a.bins[c];
    const float2 ncen = a.cen.ncen[c], cor = a.cen.cor[c];   // centred low-pass (mkid_internal.h)
    // fused last pass for X[bin]: bin = jl + NSL s,
    //   X[bin] = sum_r W_RL^{r s} W_N^{jl r} Y[jl + r NSL]   (Stockham last pass, NS = NSL)
    constexpr int RL = G::RL, NSL = G::NSL;
    const int jl = bin % NSL, sl = bin / NSL;
    float2 tl[RL - 1];
#pragma unroll
    for (int r = 1; r < RL; ++r) {
        double sn, cs;
        sincospi(-2.0 * ((double)(jl * r) / N + (double)((r * sl) % RL) / RL), &sn, &cs);
        tl[r - 1] = make_float2((float)cs, (float)sn);
    }
    const int yoff = lpad(jl);

    const int64_t k_b = (int64_t)blockIdx.x * a.frames_per_block;
    int64_t k_e = k_b + a.frames_per_block;
    if (k_e > a.K) k_e = a.K;
    if (k_b >= k_e) return;
    const int64_t k_start = k_b - kLpfHist;  // warm-up frames rebuild the low-pass history
    // outputs of this run: rows j = k_b/2 .. ; 32-bit offsets from per-run bases
    int16_t* const raw_run = a.raw + (k_b >> 1) * C;
    [[maybe_unused]] float* const phase_run = a.phase ? a.phase + (k_b >> 1) * C : nullptr;

    // prologue: hops k_start-2T+1 .. k_start+FPB-1 -> ring (slot = hop mod RS)
    {
        const int64_t h0 = k_start - 2 * T + 1;
        for (int g = 0; g < RS; g += FPB) {
            const int64_t hop = h0 + g + (tid * G::SPT) / M;
            if (hop > h0 + RS - 1) continue;
            const uint4 v = front_load<N>(a, h0 + g, tid);
            *reinterpret_cast<uint4*>(ring + (int)(((hop % RS) + RS) % RS) * M + (tid * G::SPT) % M) = v;
        }
    }
    uint4 pre = front_load<N>(a, k_start + FPB, tid);
    __syncthreads();

    // static issue priority by dispatch order (MI355X_MICROARCH.md "two waves per SIMD" item 4):
    // the later-dispatched waves of a SIMD lose every age-based arbitration and reach each barrier
    // last; raising them once before the loop trims that skew (-0.7..-1 % k_front, same-box A/B
    // profiles/r01/r01_v28_kbench_prio.json)
    {
        const int w = __builtin_amdgcn_readfirstlane(tid) / 64, nw = G::BT / 64;
        const int pr = nw >= 4 ? w * 4 / nw : 0;  // 0..3 by quarter of the workgroup
        if (pr == 1) __builtin_amdgcn_s_setprio(1);
        if (pr == 2) __builtin_amdgcn_s_setprio(2);
        if (pr == 3) __builtin_amdgcn_s_setprio(3);
    }
    float2 acc[13];
#pragma unroll
    for (int m = 0; m < 13; ++m) acc[m] = make_float2(0.f, 0.f);
    float2 ys = make_float2(0.f, 0.f);

    // 32-bit stream counters, advanced by FPB per iteration (no 64-bit modulo in the loop):
    //   rb  = ring slot of hop kb + 1 - 2T (the oldest hop frame kb reads); the FPB hops loaded
    //         for the next iteration, kb + FPB + q = (kb + 1 - 2T) + RS + q, go to slot rb + q
    //   lrow = LO-table row of frame kb;  kr = kb - k_b (frame index relative to the run)
    int rb = (int)((((k_start + 1 - 2 * T) % RS) + RS) % RS);
    int lrow = (int)((a.k0 + k_start) & (int64_t)(a.P - 1));
    const int nrun = (int)(k_e - k_b);
    const int qh = (tid * G::SPT) / M, qoff = (tid * G::SPT) % M;  // this thread's ring write

#ifdef MKID_XP_STAMPS
    int it_ = 0;
#endif
    for (int kr = -kLpfHist; kr < nrun; kr += FPB) {
        const int64_t kb = k_b + kr;
#ifdef MKID_XP_STAMPS
        ++it_;
        STAMP(14);
#endif
        // LO rows of this iteration's frames (latency hidden behind the FFT)
        float2 lov[FPB];
#pragma unroll
        for (int f = 0; f < FPB; ++f) lov[f] = (a.lo + ((lrow + f) & (a.P - 1)) * C)[c];

        // ---- PFB of frame kb + slot from the LDS ring ----
        int sb = rb + slot;
        sb -= sb >= RS ? RS : 0;
        float2 v[PTS];
#pragma unroll
        for (int r = 0; r < PTS; ++r) {
            const int p = t + r * NT;
            const int hi = p / M, off = p % M;
            // one 8-byte LDS read (a uint2 load is split into two 4-byte halves)
            const uint64_t h64 = reinterpret_cast<const uint64_t*>(hl)[p];
            const uint2 hp = make_uint2((uint32_t)h64, (uint32_t)(h64 >> 32));
            uint32_t w[T];
#pragma unroll
            for (int tau = 0; tau < T; ++tau) {
                int sl = sb + 2 * tau + hi;
                sl -= sl >= RS ? RS : 0;  // sb + 2 tau + hi < 2 RS
                w[tau] = ring[sl * M + off];
            }
            // (I_tau0 | I_tau1 << 16) etc.: low halves are I, high halves Q
            const uint32_t i01 = __builtin_amdgcn_perm(w[1], w[0], 0x05040100u);
            const uint32_t q01 = __builtin_amdgcn_perm(w[1], w[0], 0x07060302u);
            const uint32_t i23 = __builtin_amdgcn_perm(w[3], w[2], 0x05040100u);
            const uint32_t q23 = __builtin_amdgcn_perm(w[3], w[2], 0x07060302u);
            int32_t ai = dot2_i16_first(hp.x, i01);
            ai = __builtin_amdgcn_sdot2(as_s2(hp.y), as_s2(i23), ai, false);
            int32_t aq = dot2_i16_first(hp.x, q01);
            aq = __builtin_amdgcn_sdot2(as_s2(hp.y), as_s2(q23), aq, false);
            const float ur = (float)ai, ui = (float)aq;
            v[r] = make_float2(ur, ui);
            // keep the point order: stops the scheduler from hoisting all 32 ring loads at once
            // (register pressure) ...
            if ((r & 3) == 3)  // ... but let four points' loads overlap
                asm volatile("" : "+v"(v[r].x), "+v"(v[r].y), "+v"(v[r - 1].x), "+v"(v[r - 1].y),
                             "+v"(v[r - 2].x), "+v"(v[r - 2].y), "+v"(v[r - 3].x), "+v"(v[r - 3].y));
        }
        st_dft<PTS, PL::R[0]>(v);
        FSYNC(0);  // ring reads of this iteration and last iteration's select are done
        {
            int ws = rb + qh;
            ws -= ws >= RS ? RS : 0;
            *reinterpret_cast<uint4*>(ring + ws * M + qoff) = pre;
            pre = front_load<N>(a, kb + 2 * FPB, tid);
            rb += FPB;
            rb -= rb >= RS ? RS : 0;
            lrow += FPB;
        }
        st_write<N, PTS, PL::R[0], 1>(buf, v, t);
        FSYNC(1);
        st_read<N, PTS, PL::R[1]>(buf, v, t);
        FSYNC(2);
        tw2.apply(v, t);
        st_dft<PTS, PL::R[1]>(v);
        if constexpr (PL::NP == 4) {
            st_write<N, PTS, PL::R[1], G::NS2, typename G::PadB>(buf, v, t);
            FSYNC(3);
            st_read<N, PTS, PL::R[2], typename G::PadB>(buf, v, t);
            FSYNC(4);
            tw3.apply(v, t);
            st_dft<PTS, PL::R[2]>(v);
            st_write<N, PTS, PL::R[2], G::NS3>(buf, v, t);
            FSYNC(5);
        } else {
            st_write<N, PTS, PL::R[1], G::NS2>(buf, v, t);
            FSYNC(6);
        }

        // ---- select + DDC + low-pass + phase for channel c over the FPB frames ----
#pragma unroll
        for (int f = 0; f < FPB; ++f) {
            const int kf = kr + f;  // frame kb + f relative to k_b
            const float2* yf = fbuf + f * G::LDSF + yoff;
            float2 X = yf[0];
#pragma unroll
            for (int r = 1; r < RL; ++r) X = cmac(X, tl[r - 1], yf[r * NSL / 16 * 17]);
            const float2 z = cmul_add_pk(X, lov[f], ncen);   // z - c'
#ifdef MKID_XP_STAMPS
            if (f == 0) {
                asm volatile("" ::"v"(z.x), "v"(z.y));
                STAMP(12);  // frame 0 selected (its LDS reads and LO load have landed)
            }
            if (f == 2) STAMP(13);  // output 0 written
#endif
            if ((f & 1) == 0) {  // frame 2j: taps 1,3,..,25 into outputs j..j+12
#pragma unroll
                for (int m = 0; m < 13; ++m) {
                    acc[m].x = fmaf(a.taps.g[2 * m + 1], z.x, acc[m].x);
                    acc[m].y = fmaf(a.taps.g[2 * m + 1], z.y, acc[m].y);
                }
            } else {  // frame 2j+1: taps 0,2,..,24; output j complete
#pragma unroll
                for (int m = 0; m < 13; ++m) {
                    acc[m].x = fmaf(a.taps.g[2 * m], z.x, acc[m].x);
                    acc[m].y = fmaf(a.taps.g[2 * m], z.y, acc[m].y);
                }
                const float2 y = acc[0];
#pragma unroll
                for (int m = 0; m < 12; ++m) acc[m] = acc[m + 1];
                acc[12] = make_float2(0.f, 0.f);
                if (kf > 0 && kf < nrun) {
                    const int jr = (kf - 1) >> 1;  // row within the run
                    ys.x += y.x;
                    ys.y += y.y;
                    const float ph = phase_atan2(y.y + cor.y, y.x + cor.x);
                    int q = __float2int_rn(ph * 8192.0f);
                    q = q < -25736 ? -25736 : (q > 25736 ? 25736 : q);
#ifndef MKID_XP_STAMPS
                    if (phase_run) __builtin_nontemporal_store(ph, phase_run + jr * C + c);
#endif
                    __builtin_nontemporal_store((int16_t)q, raw_run + jr * C + c);
                    if (c == a.iq_ch && a.iqtap) {  // IQ snapshot tap (conv_phase_snapIQ_bram)
                        a.iqtap[2 * ((k_b >> 1) + jr)] = iq16(y.x + a.cen.tap_off.x);
                        a.iqtap[2 * ((k_b >> 1) + jr) + 1] = iq16(y.y + a.cen.tap_off.y);
                    }
                }
            }
        }
    }
    if (a.ysum) {
        ysum_add(a.ysum, c, ys.x, ys.y);
    }
}

bool fused_supported(int N) { return N == 128 || N == 256 || N == 512 || N == 1024 || N == 2048 || N == 4096; }

// the fused front end of each FFT length: k_front (this file) at N = 128 / 256, the
// wave-specialised k_front3 at 512 / 1024 / 2048 and k_front5 at 4096
hipError_t launch_fused(int N, const FrontArgs& a, hipStream_t s) {
    if (N == 4096) return launch_front5(a, s);
    if (N >= 512) return launch_front3(N, a, s);
    return launch_front(N, a, s);
}

int64_t front_hist_samples(int N) { return (int64_t)(2 * kPfbTaps - 1 + kLpfHist) * (N / 2); }

template <int N>
static hipError_t launch_front_n(const FrontArgs& a0, hipStream_t s) {
    using G = FGeo<N>;
    static std::atomic<uint64_t> attr_mask{0};
    hipError_t e = ensure_lds_attr(attr_mask, (const void*)k_front<N>, (int)G::lds_bytes);
    if (e != hipSuccess) return e;
    FrontArgs a = a0;
    if (a.K <= 0) return hipSuccess;
    // frame runs: long enough to amortise the 24-frame warm-up, enough of them to fill the CUs
    int64_t fpb = a.K / 1024;
    fpb = fpb < 64 ? 64 : (fpb > 1024 ? 1024 : fpb);
    fpb = (fpb + G::FPB - 1) / G::FPB * G::FPB;
    a.frames_per_block = fpb;
    const int64_t blocks = (a.K + fpb - 1) / fpb;
    hipLaunchKernelGGL(k_front<N>, dim3((unsigned)blocks), dim3(G::BT), G::lds_bytes, s, a);
    return hipGetLastError();
}

hipError_t launch_front(int N, const FrontArgs& a, hipStream_t s) {
    switch (N) {
        case 128: return launch_front_n<128>(a, s);
        case 256: return launch_front_n<256>(a, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace mkid
