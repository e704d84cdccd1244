// k_front5: the fused front end for N = 4096 (2048 channels, BASELINE config 5) with WAVE
// SPECIALISATION, the k_front3 scheme re-fitted to a 4096-point frame.
//
// Running every wave through both phases of an iteration (PFB + sub-FFTs, barrier, select / DDC /
// low-pass / phase, barrier; the round-2 design) keeps the FFT working set
// and two channels' low-pass state live together in 128 VGPRs (17-21 dwords spilled) and idles the
// SIMDs through both barrier phases (VALU active 45 %). Here the two phases run in different waves, one iteration
// apart, so each SIMD always holds waves of both kinds:
//   * waves 0-3 transform: wave r computes sub-FFTs r and r + 4 (512 points each, in-wave, as in
//     k_front3) of frame k and writes them to Y buffer t & 1;
//   * waves 4-15 select frame k - 1 from buffer (t - 1) & 1: waves 4-11 three channels per thread
//     (c = st + 512 q), waves 12-15 two (c = 1536 + st' + 256 q), so every SIMD carries one
//     transform wave and select work for 512 channels;
//   * one frame per iteration (the LDS does not hold two frames' Y twice at N = 4096): ring of
//     2T + 1 = 9 hops (frame k reads hops k-7 .. k; select waves 12-15 load hop k + 1 and write it
//     over hop k - 8 in the same barrier interval, off the transform chain), Y [2][8][576] float2,
//     one workgroup barrier per frame;
//   * the select threads' state lives in registers only in the select waves, so the 13 complex
//     low-pass accumulators of three channels (78 VGPRs) no longer share the file with the FFT.
// LDS: ring 72 KiB + Y 72 KiB + the channels' avgIQ sums 16 KiB = 160 KiB (the twiddles are
// computed into the transform lanes' VGPRs, and the select threads' avgIQ sums live in LDS, so
// that three channels' low-pass state fits beside the select working set in 128 VGPRs).
// Arithmetic: PFB int16 dot products, radix-8 sub-FFTs, DDC (with the centring constant fused in),
// transposed decimating low-pass, atan2, Fix16_13. The 8-way decimation combine is split (round 5):
// the transform wave that holds sub-FFTs r and r + 4 writes their radix-2 combinations
// P_r^s[k] = Y_r[k] + (-1)^s W_1024^k Y_{r+4}[k] (s = bit 9 of the bin), and a select thread reads
// the 4 regions of its bin's s and evaluates X[b] = (P_0 + t^2 P_2) + t (P_1 + t^2 P_3), t = W_N^b:
// 4 instead of 8 bin-indexed LDS reads and 4 instead of 9 complex MACs per channel-frame
// (tools/front2_layouts.py precombine_f32, same-box -6 %, profiles/r05/r05l_kbench_c5_precombine.json).
#include "front_common.h"

#include <type_traits>

#ifdef MKID_XP_STAMPS
// timing-only build: lane 0 of every wave of workgroups 0-3 stamps s_memtime at points of
// iterations (frames) 8..15 into a.phase (tools/stamps4.py ... v5); the phase output is garbage
#define STAMP5(t_, slot_)                                                                         \
    do {                                                                                          \
        __builtin_amdgcn_sched_barrier(0);                                                        \
        const uint64_t tm_ = __builtin_amdgcn_s_memtime();                                        \
        __builtin_amdgcn_sched_barrier(0);                                                        \
        if (blockIdx.x < 4 && (t_) >= 40 && (t_) < 48 && (threadIdx.x & 63) == 0)                 \
            reinterpret_cast<uint64_t*>(a.phase)[((blockIdx.x * 16 + (threadIdx.x >> 6)) * 8 +   \
                                                  ((t_) - 40)) * 16 + (slot_)] = tm_;              \
    } while (0)
#else
#define STAMP5(t_, slot_) ((void)0)
#endif

namespace mkid {

namespace {

struct G5 {
    static constexpr int N = 4096, NW = 8, M = N / 2, C = N / 2, T = kPfbTaps;
    static constexpr int BT = 1024;
    static constexpr int FW = 4;                  // transform waves
    static constexpr int SPW = NW / FW;           // sub-FFTs per transform wave per frame
    static constexpr int SPT = M / (FW * 64);     // ring-refill samples per transform thread
    static constexpr int SW = BT / 64 - FW;       // select waves
    static constexpr int SW3 = 8;                 // select waves with 3 channels per thread
    static constexpr int RS = 2 * T + 1;          // ring slots (hops)
    static constexpr int Q = M / NW;              // samples per hop plane
    static constexpr int REG = 576;               // float2 per (frame, sub-FFT) region
    static constexpr int FB = NW * REG;           // float2 per frame
    static constexpr int HIST = (2 * T - 1 + kLpfHist) * M;
    static constexpr size_t off_fbuf = (size_t)RS * M * 4;
    // [C] float2 per-channel slot: the avgIQ partial sums while the accumulator is armed
    // (k_front5<true>), else the centring constant -c' (k_front5<false>, the streaming kernel)
    static constexpr size_t off_ysum = off_fbuf + (size_t)2 * FB * 8;
    static constexpr size_t lds_bytes = off_ysum + (size_t)C * 8;
    static_assert(SPT == 8 && SPW * FW == NW, "geometry");
    static_assert(SW3 * 64 * 3 + (SW - SW3) * 64 * 2 == C, "every channel has one select slot");
    static_assert(lds_bytes <= 160 * 1024, "LDS");
};

// the 8 samples transform thread xt contributes to hop `hop` (samples 8 xt .. 8 xt + 7)
__device__ __forceinline__ void load_hop(const FrontArgs& a, int64_t hop, int xt, uint4& v0, uint4& v1) {
    const int64_t s0 = hop * G5::M + (int64_t)xt * G5::SPT;
    if (s0 >= a.K * G5::M) {
        v0 = v1 = make_uint4(0, 0, 0, 0);
        return;
    }
    if (s0 >= -a.avail) {
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 p = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a.x + s0));
        const u32x4 q = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a.x + s0 + 4));
        v0 = make_uint4(p.x, p.y, p.z, p.w);
        v1 = make_uint4(q.x, q.y, q.z, q.w);
        return;
    }
    const uint32_t* h = a.xhist + (s0 + a.avail + G5::HIST);
    v0 = *reinterpret_cast<const uint4*>(h);
    v1 = *reinterpret_cast<const uint4*>(h + 4);
}

// Pre-combination twiddles W_1024^{e + 64 r} = w0 W_16^r (w0 = W_1024^e, e = kl + 8 la), built per
// frame from w0 with three constants: u1 = w0 W_16, vv = w0 conj(W_16) (= (-i) w0 W_16^3) and
// u2 = w0 W_16^2; the odd quarter turns (-i) are applied exactly by the butterfly (add_mi / sub_mi).
// Each twiddle is within 1.1e-7 of exact (tools/front_layouts.py precombine_f32); the round-5
// recurrence wk *= W_16 reached 3.5e-7 at r = 7, and its leak of the comb's aliased bins into the
// weak channels set config 5's IQ error.
struct PreTw {
    float2 u1, vv, u2;
};
__device__ __forceinline__ PreTw pre_twiddles(float2 w0) {
    // (cos(pi/8), sin(pi/8)) and (1/sqrt(2), 1/sqrt(2)) as SGPR pairs (VOP3P takes neither a
    // literal nor a single 32-bit SGPR for its 64-bit operands); op_sel picks the half
    float a, b, h;
    asm volatile("s_mov_b32 %0, 0x3f6c835e\n\ts_mov_b32 %1, 0x3ec3ef15\n\ts_mov_b32 %2, 0x3f3504f3"
                 : "=s"(a), "=s"(b), "=s"(h));
    const uint64_t ab = tap_pair(a, b), hh = tap_pair(h, h);
    f2v m, u1, vv, u2;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(m) : "v"(f2v_of(w0)), "s"(ab));
    // u1 = (w0.x a + w0.y b, w0.y a - w0.x b), vv = (w0.x a - w0.y b, w0.y a + w0.x b)
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_hi:[1,0,0]"
        : "=v"(u1) : "v"(f2v_of(w0)), "s"(ab), "v"(m));
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_lo:[1,0,0]"
        : "=v"(vv) : "v"(f2v_of(w0)), "s"(ab), "v"(m));
    // u2 = h (w0.x + w0.y, w0.y - w0.x)
    asm("v_pk_mul_f32 %0, %1, %2" : "=v"(u2) : "v"(f2v_of(rot_1mi(w0))), "s"(hh));
    return PreTw{float2_of(u1), float2_of(vv), float2_of(u2)};
}

// hop layout: sample o at plane o % 8, plane index o / 8 stored at ring3_idx(o / 8), the paired
// plane layout of k_front3 (plane entries 64 apart adjacent, so a lane's PFB points
// r, r + 1 are one ds_read_b64)
__device__ __forceinline__ void ring_put(uint32_t* hop, int xt, uint4 v0, uint4 v1) {
    constexpr int Q = G5::Q;
    uint32_t* p = hop + ring3_idx(xt);
    p[0] = v0.x; p[Q] = v0.y; p[2 * Q] = v0.z; p[3 * Q] = v0.w;
    p[4 * Q] = v1.x; p[5 * Q] = v1.y; p[6 * Q] = v1.z; p[7 * Q] = v1.w;
}

// measured and dropped (DESIGN.md §5 k_front5): T1 in registers, LO one frame ahead, one Horner
// chain, even/odd chains, unsplit Y reads, no barrier between channels, transform-wave priority

// select / DDC / low-pass / phase of CPT channels c0 + cs q per thread, frame k - 1 of iteration t.
// Registers go to the low-pass state: the centring constants (mkid_internal.h Centring) are re-read
// per frame, -c' from the per-channel LDS slot ysl (ACC = false) or, while the avgIQ accumulator
// is armed and ysl holds its partial sums (ACC = true), from global memory; r at output frames.
// RF (waves 12-15, 256 threads like the transform waves, the lightest select work): the ring
// refill. In the barrier interval in which the transform waves compute frame k (one ahead of the
// select), hop k + 1 goes over hop k - 2T, a slot no wave reads in that interval; thread xt loads
// and writes the 8 samples load_hop / ring_put give it. Off the transform waves' chain: -8.8 %
// same box (profiles/r05/r05u_kbench_c5_refill.json; waves 4-7 or 4-11 instead: -7 %).
template <int CPT, bool ACC, bool RF>
__device__ __forceinline__ void select_run(const FrontArgs& a, const float2* fbuf, float2* ysl, int c0, int cs,
                                           int64_t k_b, int64_t k_start, int nrun, int nit, uint32_t* ring, int xt) {
    constexpr int RS = G5::RS;
    constexpr int C = G5::C;
    float2 tb[CPT];   // W_N^{bin}
    int yoff[CPT];
#pragma unroll
    for (int q = 0; q < CPT; ++q) {
        const int c = c0 + cs * q;
        const int32_t bin = a.bins[c];
        double sn, cn;
        sincospi(-2.0 * (double)bin / G5::N, &sn, &cn);
        tb[q] = make_float2((float)cn, (float)sn);
        // P_r^s of the bin's half s = bit 9 (regions r + 4 s, r = 0..3): see the transform waves
        yoff[q] = yswz(bin & 511) + ((bin >> 9) & 1) * 4 * G5::REG;
        ysl[c] = ACC ? make_float2(0.f, 0.f) : a.cen.ncen[c];   // the thread's own channels only
    }
    uint64_t gp[13];
#pragma unroll
    for (int m = 0; m < 13; ++m) gp[m] = tap_pair(a.taps.g[2 * m], a.taps.g[2 * m + 1]);
    float2 acc[CPT][13];
#pragma unroll
    for (int q = 0; q < CPT; ++q)
#pragma unroll
        for (int m = 0; m < 13; ++m) acc[q][m] = make_float2(0.f, 0.f);
    int16_t* const raw_run = a.raw + (k_b >> 1) * C;
    float* const phase_run = a.phase ? a.phase + (k_b >> 1) * C : nullptr;
    int lrow = (int)((a.k0 + k_start) & (int64_t)(a.P - 1));
    __syncthreads();   // prologue: ring written
    if (RF) {          // transform iteration 0 computes frame k_start: hop k_start + 1
        uint4 v0, v1;
        const int64_t h = k_start + 1;
        load_hop(a, h, xt, v0, v1);
        ring_put(ring + (int)(((h % RS) + RS) % RS) * G5::M, xt, v0, v1);
    }
    __syncthreads();   // transform iteration 0 (frame k_start) wrote Y buffer 0
    // frames in pairs (even: accumulate, odd: output), one barrier after each: frame k_start + 2p
    // is in Y buffer 0, k_start + 2p + 1 in buffer 1 (nit is even). Unrolled by hand so the
    // accumulators keep their registers (as a parity branch, the two paths' results met in phis that
    // the allocator resolved with copies and ~20 spilled accumulators).
    // the warm-up pairs (no output) and the output pairs are separate loops, so that every store of
    // the output loop is unconditional and the waits on loads issued before it are counted exactly
    auto pair = [&](int p, auto outc) {
        constexpr bool OUTF = decltype(outc)::value;
        const int kf = -kLpfHist + 2 * p;   // even
#pragma unroll
        for (int f = 0; f < 2; ++f) {
            STAMP5(2 * p + 1 + f, 8);
            // this interval's refill (transform iteration 2p + f + 1, frame k_start + 2p + f + 1):
            // hop k_start + 2p + f + 2, loaded first (its wait then covers nothing issued later)
            const int64_t hr = k_start + 2 * p + f + 2;
            const bool rf = RF && 2 * p + f + 1 < nit;
            uint4 rv0, rv1;
            if (rf) load_hop(a, hr, xt, rv0, rv1);
            // channel base re-defined every frame so per-channel addresses are rebuilt in the loop
            // (a few VALU) instead of being hoisted as 64-bit pointers that crowd the low-pass state
            int cb = c0;
            asm volatile("" : "+v"(cb));
            const float2* yf = fbuf + f * G5::FB;
            // the LO row of this frame is loaded at the frame's start (loading it a frame ahead was
            // measured flat, DESIGN.md §5 k_front5); the centres of an output frame likewise
            float2 lov[CPT], ncv[CPT];
            {
                const char* lorow = reinterpret_cast<const char*>(a.lo + ((lrow + f) & (a.P - 1)) * C);
                const char* ncrow = reinterpret_cast<const char*>(a.cen.ncen);
#pragma unroll
                for (int q = 0; q < CPT; ++q) {
                    lov[q] = *reinterpret_cast<const float2*>(lorow + (uint32_t)(cb + cs * q) * 8u);
                    ncv[q] = ACC ? *reinterpret_cast<const float2*>(ncrow + (uint32_t)(cb + cs * q) * 8u)
                                 : ysl[cb + cs * q];
                }
            }
            [[maybe_unused]] float2 corv[CPT];
            if (f == 1) {
                const char* corow = reinterpret_cast<const char*>(a.cen.cor);
#pragma unroll
                for (int q = 0; q < CPT; ++q) corv[q] = *reinterpret_cast<const float2*>(corow + (uint32_t)(cb + cs * q) * 8u);
            }
            auto zq = [&](int q) {   // z - c' of channel slot q
                const float2 lo = lov[q];
                const float2* yq = yf + yoff[q];
                // X[b] = sum_r t^r P_r^s[b mod 512], t = W_N^b: (P0 + t^2 P2) + t (P1 + t^2 P3)
                const float2 y0 = yq[0], y1 = yq[G5::REG], y2 = yq[2 * G5::REG], y3 = yq[3 * G5::REG];
                const float2 t2 = cmul_pk(tb[q], tb[q]);
                const float2 xa = cmac(y0, t2, y2), xb = cmac(y1, t2, y3);
                return cmul_add_pk(cmac(xa, tb[q], xb), lo, ncv[q]);
            };
            if (f == 0) {
                // every channel's X first (its 4 reads in flight together), then the accumulations
                float2 zz[CPT];
#pragma unroll
                for (int q = 0; q < CPT; ++q) zz[q] = zq(q);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int q = 0; q < CPT; ++q) {
#pragma unroll
                    for (int m = 0; m < 13; ++m) acc[q][m] = fma_tap<1>(gp[m], zz[q], acc[q][m]);   // g_{2m+1}
                }
            } else {
                const int ko = kf + 1;   // odd: output row (ko - 1) / 2 of the run
                constexpr bool out = OUTF;   // ko > 0 && ko < nrun
                const int jr = (ko - 1) >> 1;
                // every channel's phase first, then the frame's stores: a load waited on after a
                // store would wait for the store too (vmcnt retires in order)
                float ph[CPT];
                uint32_t iqv = 0;
                bool iqhit = false;
#pragma unroll
                for (int q = 0; q < CPT; ++q) {
                    const float2 z = zq(q);
                    const float2 y = fma_tap<0>(gp[0], z, acc[q][0]);                                // g_0
#pragma unroll
                    for (int m = 0; m < 12; ++m) acc[q][m] = fma_tap<0>(gp[m + 1], z, acc[q][m + 1]);  // g_{2m+2}
                    acc[q][12] = make_float2(0.f, 0.f);
                    ph[q] = phase_atan2(y.y + corv[q].y, y.x + corv[q].x);
                    if (out) {
                        const int c = cb + cs * q;
                        // avgIQ only while the accumulator is armed (mkid_set_accumulator; the
                        // reference accumulates on demand, startAccumulator / avgIQ_ctrl,
                        // ROACH_Setup.py:654-659). One owner per entry: a plain read-add-write (LDS
                        // float atomics stalled every wave's LDS traffic on output frames)
                        if (ACC) {
                            float2 ysv = ysl[c];
                            ysv.x += y.x;
                            ysv.y += y.y;
                            ysl[c] = ysv;
                        }
                        if (a.iqtap) {               // uniform; the IQ-tap channel's sample by select
                            const bool hit = c == a.iq_ch;
                            const float2 yt = make_float2(y.x + a.cen.tap_off.x, y.y + a.cen.tap_off.y);
                            const uint32_t v = (uint32_t)(uint16_t)iq16(yt.x) | ((uint32_t)(uint16_t)iq16(yt.y) << 16);
                            iqv = hit ? v : iqv;
                            iqhit = iqhit || hit;
                        }
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
                if (out) {
                    // uniform row bases + 32-bit lane offsets (SGPR-base stores, no 64-bit VGPR pointers)
                    char* const prow = reinterpret_cast<char*>(phase_run + jr * C);
                    char* const rrow = reinterpret_cast<char*>(raw_run + jr * C);
#pragma unroll
                    for (int q = 0; q < CPT; ++q) {
                        const uint32_t c = (uint32_t)(cb + cs * q);
                        int qv = __float2int_rn(ph[q] * 8192.0f);
                        qv = qv < -25736 ? -25736 : (qv > 25736 ? 25736 : qv);
#ifndef MKID_XP_STAMPS
                        if (phase_run) __builtin_nontemporal_store(ph[q], reinterpret_cast<float*>(prow + c * 4u));
#endif
                        __builtin_nontemporal_store((int16_t)qv, reinterpret_cast<int16_t*>(rrow + c * 2u));
                    }
                    if (iqhit) *reinterpret_cast<uint32_t*>(a.iqtap + 2 * ((k_b >> 1) + jr)) = iqv;
                }
            }
            if (rf) ring_put(ring + (int)(((hr % RS) + RS) % RS) * G5::M, xt, rv0, rv1);
            STAMP5(2 * p + 1 + f, 9);
            __syncthreads();   // Y buffer f read; the transform waves wrote the next frame into 1 - f
            STAMP5(2 * p + 1 + f, 10);
        }
        lrow += 2;
    };
    for (int p = 0; p < kLpfHist / 2; ++p) pair(p, std::false_type{});
    for (int p = kLpfHist / 2; p < nit / 2; ++p) pair(p, std::true_type{});
    if (ACC)
#pragma unroll
        for (int q = 0; q < CPT; ++q) {
            const float2 ys = ysl[c0 + cs * q];
            ysum_add(a.ysum, c0 + cs * q, ys.x, ys.y);
        }
}

}  // namespace

template <bool ACC>
__global__ __launch_bounds__(G5::BT, 4) void k_front5(FrontArgs a) {
    using G = G5;
    constexpr int NW = G::NW, M = G::M, T = G::T, RS = G::RS;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t* ring = reinterpret_cast<uint32_t*>(smem);
    float2* fbuf = reinterpret_cast<float2*>(smem + G::off_fbuf);
    float2* ysl = reinterpret_cast<float2*>(smem + G::off_ysum);

    const int tid = threadIdx.x;
    const int L = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

    const int64_t k_b = (int64_t)blockIdx.x * a.frames_per_block;
    int64_t k_e = k_b + a.frames_per_block;
    if (k_e > a.K) k_e = a.K;
    if (k_b >= k_e) return;
    const int64_t k_start = k_b - kLpfHist;
    const int nrun = (int)(k_e - k_b);
    const int nit = nrun + kLpfHist;                 // iterations: frames k_start .. k_e - 1 (even)

#ifdef MKID_XP_STAMPS
    uint64_t* const bst = reinterpret_cast<uint64_t*>(a.phase) + 8192 + 4 * blockIdx.x;   // per-block stamps
    if (tid == 0) {
        bst[0] = __builtin_amdgcn_s_memtime();
        bst[2] = (uint64_t)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));   // HW_ID
    }
#endif
    if (wave < G::FW) {
        // ---------------- transform waves: sub-FFTs rw + FW s of frame k_start + t ----------------
        const int rw = wave, xt = tid;               // xt: thread among the transform waves
        {   // prologue: hops k_start-2T+1 .. k_start -> ring (slot = hop mod RS)
            const int64_t h0 = k_start - 2 * T + 1;
            for (int g = 0; g < 2 * T; ++g) {
                uint4 v0, v1;
                load_hop(a, h0 + g, xt, v0, v1);
                ring_put(ring + (int)((((h0 + g) % RS) + RS) % RS) * M, xt, v0, v1);
            }
        }
        uint2 tq[G::SPW][8];
#pragma unroll
        for (int s = 0; s < G::SPW; ++s)
#pragma unroll
            for (int r = 0; r < 8; ++r) tq[s][r] = a.pfbq[NW * (64 * r + L) + rw + G::FW * s];
        const int la = L & 7, kl = L >> 3;
        int rb = (int)((((k_start + 1 - 2 * T) % RS) + RS) % RS);   // slot of hop k - 2T + 1
        __syncthreads();
        // the lane's stage-1 / stage-2 twiddles W_512^{L k}, W_64^{la k} (the same every frame)
        float2 w1[7], w2[7];
        float2 w0;   // W_1024^{kl + 8 la} (the pre-combination twiddle of output 0)
        {
            double sn, cn;
            sincospi(-2.0 * (double)(kl + 8 * la) / 1024.0, &sn, &cn);
            w0 = make_float2((float)cn, (float)sn);
        }
#pragma unroll
        for (int k = 1; k < 8; ++k) {
            double sn, cn;
            sincospi(-2.0 * (double)(L * k) / 512.0, &sn, &cn);
            w1[k - 1] = make_float2((float)cn, (float)sn);
            sincospi(-2.0 * (double)(la * k) / 64.0, &sn, &cn);
            w2[k - 1] = make_float2((float)cn, (float)sn);
            asm volatile("" : "+v"(w1[k - 1].x), "+v"(w1[k - 1].y), "+v"(w2[k - 1].x), "+v"(w2[k - 1].y));
        }
        for (int t = 0; t <= nit; ++t) {
            STAMP5(t, 0);
            if (t < nit) {
                float2* fb = fbuf + (t & 1) * G::FB;
                // Y_rw of sub-FFT 0, held in VGPRs for the pre-combination (16 VGPRs the transform
                // path has since the ring refill left it; -3 % against its LDS write + read-back,
                // profiles/r05/r05z_kbench_c5_yreg.json)
                float2 yr[8];
#pragma unroll
                for (int s = 0; s < G::SPW; ++s) {
                    const int w = rw + G::FW * s;
                    float2* reg = fb + w * G::REG;
                    uint32_t xr[8][T];
#pragma unroll
                    for (int hi = 0; hi < 2; ++hi)
#pragma unroll
                        for (int tau = 0; tau < T; ++tau) {
                            int sl = rb + 2 * tau + hi;
                            sl -= sl >= RS ? RS : 0;
                            const uint32_t* pl = ring + sl * M + w * G::Q + 2 * L;
                            const uint2 p01 = *reinterpret_cast<const uint2*>(pl);
                            const uint2 p23 = *reinterpret_cast<const uint2*>(pl + 128);
                            xr[4 * hi + 0][tau] = p01.x;
                            xr[4 * hi + 1][tau] = p01.y;
                            xr[4 * hi + 2][tau] = p23.x;
                            xr[4 * hi + 3][tau] = p23.y;
                        }
                    float2 v[8];
#pragma unroll
                    for (int r = 0; r < 8; ++r) {
                        const uint32_t* x4 = xr[r];
                        const uint32_t i01 = __builtin_amdgcn_perm(x4[1], x4[0], kPermI);
                        const uint32_t q01 = __builtin_amdgcn_perm(x4[1], x4[0], kPermQ);
                        const uint32_t i23 = __builtin_amdgcn_perm(x4[3], x4[2], kPermI);
                        const uint32_t q23 = __builtin_amdgcn_perm(x4[3], x4[2], kPermQ);
                        int32_t ai = dot2_first(tq[s][r].x, i01);
                        ai = __builtin_amdgcn_sdot2(as_s2(tq[s][r].y), as_s2(i23), ai, false);
                        int32_t aq = dot2_first(tq[s][r].x, q01);
                        aq = __builtin_amdgcn_sdot2(as_s2(tq[s][r].y), as_s2(q23), aq, false);
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
                    if (s == 0) {
#pragma unroll
                        for (int r = 0; r < 8; ++r) yr[r] = v[r];   // Y_rw, combined below
                    } else {
                        // radix-2 pre-combination of this wave's two sub-FFTs (w = rw + 4):
                        //   P_rw^s[k] = Y_rw[k] + (-1)^s W_1024^k Y_{rw+4}[k],  k = 64 r + kl + 8 la
                        // (W_N^{4b} = W_1024^k (-1)^{b >> 9}), so a select reads 4 regions, not 8
                        float2* yw0 = fb + rw * G::REG + ((kl + 8 * la) ^ (la << 1));
                        float2 w0f = w0;   // the twiddles are rebuilt per frame, not held
                        asm volatile("" : "+v"(w0f.x), "+v"(w0f.y));
                        const PreTw pt = pre_twiddles(w0f);
#pragma unroll
                        for (int r = 0; r < 8; ++r) {
                            // W_1024^{64 r + e}: w0, u1, u2, (-i) vv, (-i) w0, (-i) u1, (-i) u2, -vv
                            const float2 wk = (r & 3) == 0 ? w0f : ((r & 3) == 1 ? pt.u1 : ((r & 3) == 2 ? pt.u2 : pt.vv));
                            const float2 y0 = yr[r];
                            const float2 e = cmul_pk(v[r], wk);
                            float2 p, q;
                            if (r < 3) {
                                p = cadd(y0, e);
                                q = csub(y0, e);
                            } else if (r < 7) {          // d = (-i) e
                                p = add_mi(y0, e);
                                q = sub_mi(y0, e);
                            } else {                     // d = -e
                                p = csub(y0, e);
                                q = cadd(y0, e);
                            }
                            yw0[64 * r] = p;
                            yw[64 * r] = q;
                        }
                    }
                    STAMP5(t, 1 + s);
                }
                // the ring refill (hop k + 1 over hop k - 2T) is done by select waves 12-15
                rb += 1;
                rb -= rb >= RS ? RS : 0;
            }
            STAMP5(t, 3);
            __syncthreads();
            STAMP5(t, 4);
        }
#ifdef MKID_XP_STAMPS
        if (tid == 0) bst[1] = __builtin_amdgcn_s_memtime();
#endif
    } else {
        // ---------------- select waves, one frame behind the transform waves --------------------
        const int sw = wave - G::FW;
        if (sw < G::SW3)
            select_run<3, ACC, false>(a, fbuf, ysl, sw * 64 + L, 512, k_b, k_start, nrun, nit, ring, 0);
        else
            select_run<2, ACC, true>(a, fbuf, ysl, 3 * 512 + (sw - G::SW3) * 64 + L, 256, k_b, k_start, nrun, nit,
                                     ring, tid - (G::FW + G::SW3) * 64);
    }
}

hipError_t launch_front5(const FrontArgs& a0, hipStream_t s) {
    static std::atomic<uint64_t> attr_mask{0}, attr_mask_acc{0};
    const void* fn = a0.ysum ? (const void*)k_front5<true> : (const void*)k_front5<false>;
    hipError_t e = ensure_lds_attr(a0.ysum ? attr_mask_acc : attr_mask, fn, (int)G5::lds_bytes);
    if (e != hipSuccess) return e;
    FrontArgs a = a0;
    if (a.K <= 0) return hipSuccess;
    // one run per CU (a 2^30-sample chunk: 2048 frames per CU of MI355X's 256, the 24-frame
    // low-pass warm-up 1.2 % of it); runs are even so that every run starts on an output row
    const int64_t ncu = a.ncu > 0 ? a.ncu : 256;
    int64_t fpb = a.K / ncu;
    fpb = fpb < 64 ? 64 : (fpb > 4096 ? 4096 : fpb);
    fpb = (fpb + 1) / 2 * 2;
    a.frames_per_block = fpb;
    const int64_t blocks = (a.K + fpb - 1) / fpb;
    if (a.ysum)
        hipLaunchKernelGGL(k_front5<true>, dim3((unsigned)blocks), dim3(G5::BT), G5::lds_bytes, s, a);
    else
        hipLaunchKernelGGL(k_front5<false>, dim3((unsigned)blocks), dim3(G5::BT), G5::lds_bytes, s, a);
    return hipGetLastError();
}

}  // namespace mkid
