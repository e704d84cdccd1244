// Fused front end v2 (N = 512, 1024, 2048): K1-K6 in one pass over the ADC stream, with an
// FFT that exchanges data between waves ONCE per frame and two workgroup barriers per iteration
// (v1, k_front.hip: three cross-wave LDS exchanges, six barriers).
//
// Decimation in time by NW = N/512: X[k] = sum_{w<NW} W_N^{w k} Y_w[k mod 512], where Y_w is the
// 512-point DFT of u[NW m + w]. Wave w of a frame computes Y_w entirely inside the wave:
//   lane L (0..63) holds v[r] = u[NW (64 r + L) + w], r = 0..7 (computed by the PFB straight from
//   the LDS ring), then
//   stage 1  radix-8 over r;            twiddle W_512^{L k}
//   T1       register bits <-> lane bits 3-5: DPP row_ror:8 with bank masks (bit 3),
//            v_permlane16_swap (bit 4), v_permlane32_swap (bit 5) -- VALU only, no LDS
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
//   ring   RS hops of M samples; sample offset o of a hop at (o % NW) (M / NW) + o / NW, so the
//          PFB's reads of points NW (64 r + L) + w are consecutive in L
//   taps   point p at (p % NW) 512 + p / NW, int16 quads (8 B)
//   region per (frame, wave): 576 float2; T2 uses i + (i >> 3), Y uses k ^ ((k >> 2) & 14)
#include "fft_common.h"
#include "mkid_internal.h"

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

#ifndef MKID_NT_LOADS
#define MKID_NT_LOADS 1
#endif
#ifndef MKID_NT_STORES
#define MKID_NT_STORES 1
#endif

#ifndef MKID_CMUL
#define MKID_CMUL cmul_pk
#endif
#ifndef MKID_F2_PAIRRING
#define MKID_F2_PAIRRING 1
#endif
#ifndef MKID_F2_T1LDS
#define MKID_F2_T1LDS 1
#endif
// PFB tap quads in VGPRs (16 per lane; -1.1 % k_front2 same-box, profiles/r02_v11_kbench_f2_tapreg.json)
#ifndef MKID_F2_TAPREG
#define MKID_F2_TAPREG 1
#endif

namespace mkid {

namespace {

typedef short fshort2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ fshort2_t as_s2(uint32_t v) { return __builtin_bit_cast(fshort2_t, v); }
__device__ __forceinline__ int32_t dot2_first(uint32_t h, uint32_t x) {
    int32_t d;
    asm("v_dot2_i32_i16 %0, %1, %2, 0" : "=v"(d) : "v"(h), "v"(x));
    return d;
}

template <int N>
struct G2 {
    static constexpr int NW = N / 512;                 // waves (512-point sub-FFTs) per frame
    static constexpr int FPB = 4;                      // frames per iteration
    static constexpr int BT = FPB * NW * 64;           // threads == channels
    static constexpr int M = N / 2, C = N / 2, T = kPfbTaps;
    static constexpr int RS = 2 * T - 1 + FPB;         // ring slots (hops)
    static constexpr int REG = 576;                    // float2 per (frame, wave) region
    static constexpr int FB = NW * REG;                // float2 per frame
    static constexpr int HIST = (2 * T - 1 + kLpfHist) * M;
    static constexpr size_t off_fbuf = (size_t)RS * M * 4;
    static constexpr size_t off_taps = off_fbuf + (size_t)FPB * FB * 8;
    static constexpr size_t off_tw1 = off_taps + (size_t)N * 8;      // W_512^{L k}: [k-1][L]
    static constexpr size_t off_tw2 = off_tw1 + (size_t)7 * 64 * 8;  // W_64^{l k}: [k-1][l]
    static constexpr size_t lds_bytes = off_tw2 + (size_t)7 * 8 * 8;
    static_assert(BT == C, "one channel per thread");
    static_assert(N >= 512 && N <= 2048, "v2 geometry");
};

// 16 bytes (4 samples) this thread contributes to the FPB hops starting at first_hop
template <int N>
__device__ __forceinline__ uint4 load4(const FrontArgs& a, int64_t first_hop, int tid) {
    using G = G2<N>;
    const int64_t s0 = first_hop * G::M + (int64_t)tid * 4;
    if (s0 >= a.K * G::M) return make_uint4(0, 0, 0, 0);
#if MKID_NT_LOADS
    if (s0 >= -a.avail) {
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a.x + s0));
        return make_uint4(v.x, v.y, v.z, v.w);
    }
#else
    if (s0 >= -a.avail) return *reinterpret_cast<const uint4*>(a.x + s0);
#endif
    return *reinterpret_cast<const uint4*>(a.xhist + (s0 + a.avail + G::HIST));
}

// samples qoff..qoff+3 of a hop (qoff a multiple of 4) into the permuted hop layout
template <int N>
__device__ __forceinline__ void ring_put(uint32_t* hop, int qoff, uint4 v) {
    using G = G2<N>;
    constexpr int Q = G::M / G::NW;
    if constexpr (G::NW == 1) {
        *reinterpret_cast<uint4*>(hop + qoff) = v;
    } else if constexpr (G::NW == 2) {
        *reinterpret_cast<uint2*>(hop + qoff / 2) = make_uint2(v.x, v.z);
        *reinterpret_cast<uint2*>(hop + Q + qoff / 2) = make_uint2(v.y, v.w);
    } else {
        hop[qoff / 4] = v.x;
        hop[Q + qoff / 4] = v.y;
        hop[2 * Q + qoff / 4] = v.z;
        hop[3 * Q + qoff / 4] = v.w;
    }
}

// T1: swap register bit i with lane bit 3 + i (i = 0, 1, 2). v_mov_b32_dpp row_ror:8 reads lane
// ^ 8 within each row of 16; lanes of disabled banks (4 lanes each) keep `old`.
template <int BANKS>
__device__ __forceinline__ float upd_ror8(float old, float src) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, old),
                                                                 __builtin_bit_cast(int, src), 0x128, 0xf,
                                                                 BANKS, false));
}

[[maybe_unused]] __device__ __forceinline__ void t1_transpose(float2 (&v)[8]) {
    // register bit 0 <-> lane bit 3: lanes 8-15 of every row (banks 2, 3) take the partner
    // register of lane ^ 8; lanes 0-7 (banks 0, 1) the other way round (row_ror:8 = lane ^ 8)
#pragma unroll
    for (int r0 = 0; r0 < 8; r0 += 2) {
        const float2 a0 = v[r0], a1 = v[r0 + 1];
        v[r0].x = upd_ror8<0xC>(a0.x, a1.x);
        v[r0].y = upd_ror8<0xC>(a0.y, a1.y);
        v[r0 + 1].x = upd_ror8<0x3>(a1.x, a0.x);
        v[r0 + 1].y = upd_ror8<0x3>(a1.y, a0.y);
    }
    // register bit 1 <-> lane bit 4: v_permlane16_swap (odd rows of x <-> even rows of y)
    constexpr int kP16[4] = {0, 1, 4, 5};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r0 = kP16[i];
        const auto sx = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(int, v[r0].x),
                                                         __builtin_bit_cast(int, v[r0 + 2].x), false, false);
        const auto sy = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(int, v[r0].y),
                                                         __builtin_bit_cast(int, v[r0 + 2].y), false, false);
        v[r0] = make_float2(__builtin_bit_cast(float, (int)sx[0]), __builtin_bit_cast(float, (int)sy[0]));
        v[r0 + 2] = make_float2(__builtin_bit_cast(float, (int)sx[1]), __builtin_bit_cast(float, (int)sy[1]));
    }
    // register bit 2 <-> lane bit 5: v_permlane32_swap (upper half of x <-> lower half of y)
#pragma unroll
    for (int r0 = 0; r0 < 4; ++r0) {
        const auto sx = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(int, v[r0].x),
                                                         __builtin_bit_cast(int, v[r0 + 4].x), false, false);
        const auto sy = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(int, v[r0].y),
                                                         __builtin_bit_cast(int, v[r0 + 4].y), false, false);
        v[r0] = make_float2(__builtin_bit_cast(float, (int)sx[0]), __builtin_bit_cast(float, (int)sy[0]));
        v[r0 + 4] = make_float2(__builtin_bit_cast(float, (int)sx[1]), __builtin_bit_cast(float, (int)sy[1]));
    }
}

__device__ __forceinline__ int yswz(int k) { return k ^ ((k >> 2) & 14); }

// k_front3 ring plane layout (N = 2048, NW = 4, Q = 256 samples per plane): plane index
// i = 64 j + l (j = 0..3) is stored at 128 (j >> 1) + 2 l + (j & 1), so the PFB's points j and
// j + 1 of a lane are one ds_read_b64 (16 reads of 8 B per sub-FFT instead of 32 of 4 B;
// conflict-free: 32 lanes x 2 dwords). The refill's ds_write_b32 become 2-way bank conflicts,
// which cost no extra cycles for ds_write_b32 (MI355X_MICROARCH.md §LDS).
__device__ __forceinline__ int ring3_idx(int i) { return 128 * (i >> 7) + 2 * (i & 63) + ((i >> 6) & 1); }
__device__ __forceinline__ void ring3_put(uint32_t* hop, int qoff, uint4 v) {
    constexpr int Q = 256;
    const int a = ring3_idx(qoff / 4);
    hop[a] = v.x;
    hop[Q + a] = v.y;
    hop[2 * Q + a] = v.z;
    hop[3 * Q + a] = v.w;
}

// the same paired plane layout for any NW (every plane is Q = M / NW = 256 samples): samples
// qoff..qoff+3 of a hop go to plane (o mod NW), plane index o / NW (qoff is a multiple of 4, so the
// 4 indices of a plane stay in one 64-block and ring3_idx steps by 2)
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
        ring3_put(hop, qoff, v);
    }
}

// T1 through the wave's own LDS region instead of DPP/permlane moves: element (lane 8 kl + la,
// register r) goes to (lane 8 r + la, register kl). Lane L writes register r at 72 r + L; lane L'
// reads register r' at 72 (L' >> 3) + 8 r' + (L' & 7). Both patterns are bank-conflict-free for
// ds_*_b64 (writes: 32 consecutive entries; reads: entries 8 (r + r') + la mod 32 distinct over a
// lane group, r = L' >> 3 < 4 there), every offset an immediate. 8 writes + 8 reads replace 32
// VALU cross-lane moves (the transform waves are VALU-issue-bound).
__device__ __forceinline__ void t1_lds(float2 (&v)[8], float2* reg, int L) {
#pragma unroll
    for (int r = 0; r < 8; ++r) reg[72 * r + L] = v[r];
    __builtin_amdgcn_wave_barrier();
    const float2* rd = reg + 72 * (L >> 3) + (L & 7);
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] = rd[8 * r];
    __builtin_amdgcn_wave_barrier();
}

}  // namespace

template <int N>
__global__ __launch_bounds__(G2<N>::BT, 4) void k_front2(FrontArgs a) {
    using G = G2<N>;
    constexpr int NW = G::NW, M = G::M, C = G::C, T = G::T, RS = G::RS, FPB = G::FPB;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t* ring = reinterpret_cast<uint32_t*>(smem);
    float2* fbuf = reinterpret_cast<float2*>(smem + G::off_fbuf);
    [[maybe_unused]] const uint2* taps = reinterpret_cast<const uint2*>(smem + G::off_taps);
    float2* tw1 = reinterpret_cast<float2*>(smem + G::off_tw1);
    float2* tw2 = reinterpret_cast<float2*>(smem + G::off_tw2);

    const int tid = threadIdx.x;
    const int L = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int slot = wave / NW;   // frame of the iteration this wave transforms
    const int w = wave % NW;      // its sub-FFT
    float2* reg = fbuf + slot * G::FB + w * G::REG;

    // tables: taps in the permuted point order, stage-1/2 twiddles
    if (!MKID_F2_TAPREG)
        for (int p = tid; p < N; p += G::BT) reinterpret_cast<uint2*>(smem + G::off_taps)[(p % NW) * 512 + p / NW] = a.pfbq[p];
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
            const uint4 v = load4<N>(a, h0 + g, tid);
#if MKID_F2_PAIRRING
            ring_put_paired<N>(ring + (int)(((hop % RS) + RS) % RS) * M, qoff, v);
#else
            ring_put<N>(ring + (int)(((hop % RS) + RS) % RS) * M, qoff, v);
#endif
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
#if !MKID_F2_TAPREG
    const uint2* tp = taps + w * 512 + L;     // tap quad of point r at tp[64 r]
#else
    // the wave's points are the same every frame: tap quads in VGPRs instead of LDS reads
    uint2 tq[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) tq[r] = a.pfbq[NW * (64 * r + L) + w];
#endif
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
        const uint4 pre = load4<N>(a, k_b + kr + FPB, tid);
        float2 lov[FPB];
#pragma unroll
        for (int f = 0; f < FPB; ++f) lov[f] = (a.lo + ((lrow + f) & (a.P - 1)) * C)[c];

        // ---- PFB: points NW (64 r + L) + w of frame kb + slot ----
        int sb = rb + slot;
        sb -= sb >= RS ? RS : 0;
        float2 v[8];
        [[maybe_unused]] uint32_t xo[T];   // MKID_F2_PAIRRING: the odd point's samples
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const int hi = r >> 2;
            const int pos = w * (M / NW) + 64 * (r & 3) + L;
#if MKID_F2_TAPREG
            const uint64_t h64 = (uint64_t)tq[r].x | ((uint64_t)tq[r].y << 32);
#else
            const uint64_t h64 = *reinterpret_cast<const uint64_t*>(tp + 64 * r);
#endif
            uint32_t x4[T];
#if MKID_F2_PAIRRING
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
            (void)pos;
#else
#pragma unroll
            for (int tau = 0; tau < T; ++tau) {
                int sl = sb + 2 * tau + hi;
                sl -= sl >= RS ? RS : 0;
                x4[tau] = ring[sl * M + pos];
            }
#endif
            const uint32_t i01 = __builtin_amdgcn_perm(x4[1], x4[0], 0x05040100u);
            const uint32_t q01 = __builtin_amdgcn_perm(x4[1], x4[0], 0x07060302u);
            const uint32_t i23 = __builtin_amdgcn_perm(x4[3], x4[2], 0x05040100u);
            const uint32_t q23 = __builtin_amdgcn_perm(x4[3], x4[2], 0x07060302u);
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
        for (int k = 1; k < 8; ++k) v[k] = MKID_CMUL(v[k], t1[64 * (k - 1)]);
        // ---- T1 (through the wave's own LDS region, or VALU cross-lane) + stage 2 + twiddle ----
#if MKID_F2_T1LDS
        t1_lds(v, reg, L);
#else
        t1_transpose(v);
#endif
        dft<8>(v);
#pragma unroll
        for (int k = 1; k < 8; ++k) v[k] = MKID_CMUL(v[k], t2[8 * (k - 1)]);
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
#if MKID_F2_PAIRRING
            ring_put_paired<N>(ring + ws * M, qoff, pre);
#else
            ring_put<N>(ring + ws * M, qoff, pre);
#endif
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
            const float2 z = MKID_CMUL(X, lov[f]);
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
#if MKID_NT_STORES
                    if (phase_run) __builtin_nontemporal_store(ph, phase_run + jr * C + c);
#else
                    if (phase_run) (phase_run + jr * C)[c] = ph;
#endif
#endif
#if MKID_NT_STORES
                    __builtin_nontemporal_store((int16_t)q, raw_run + jr * C + c);
#else
                    (raw_run + jr * C)[c] = (int16_t)q;
#endif
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


// ---------------------------------------------------------------------------------------------
// k_front3 (N = 2048, config 3): the k_front2 arithmetic with WAVE SPECIALISATION. In k_front2
// every wave runs the FFT phase, then every wave runs the select phase, with a workgroup barrier
// between them: when all four waves of a SIMD wait on LDS (ring reads, the select's bin-indexed
// reads) or on a barrier, the SIMD idles (stamps: the FFT phase of the last wave of a SIMD ends
// ~2.4k cycles after the first, VALU busy ~70 %). Here waves 0-7 only transform (2 frames per
// iteration, one 512-point sub-FFT each) and waves 8-15 only select / mix / low-pass / phase
// (two channels per thread), one iteration behind, on a double-buffered Y: each SIMD holds two
// FFT and two select waves whose LDS waits and VALU bursts interleave, one barrier per iteration.
//   ring  RS = 2T - 1 + 2F hops: iteration t reads hops k-7 .. k+1 (frames k, k+1) while its
//         FFT waves write hops k+2, k+3 (prefetched at the loop top) over hops k-9, k-8
//   Y     [2][F][NW][576] float2, iteration t writes buffer t & 1, its select reads (t - 1) & 1
// Registers: the FFT path holds the PFB taps and the 512-point sub-FFT, the select path two
// channels' low-pass state; branches are wave-uniform, so the two live sets do not add up.
#ifndef MKID_F3_T1LDS
#define MKID_F3_T1LDS 1
#endif
#ifndef MKID_F3_TWREG
#define MKID_F3_TWREG 1
#endif
#ifndef MKID_F3_PAIRRING
#define MKID_F3_PAIRRING 1
#endif
// MKID_F3_DECOUPLE: no workgroup barrier in the loop. The transform waves meet each other through an
// LDS arrival counter (the ring refill of iteration t is read by all of them in t + 1) and the two
// groups hand Y over through a second one, on THREE Y buffers: transform t may run while the select
// waves are still on t - 2, so a slow wave of one group no longer stalls the other every iteration
// (stamps with the barrier: both groups waited ~700-900 cycles per iteration at ~3.0k of work).
#ifndef MKID_F3_DECOUPLE
#define MKID_F3_DECOUPLE 0
#endif

#ifndef MKID_F3_SLEEP
#define MKID_F3_SLEEP 1
#endif
// LDS progress words. The transform waves share one arrival counter: a wave starts iteration t only
// once it reads 8 t, so no transform wave is more than one iteration ahead of another and "counter
// >= 8 t" means every one of them finished t - 1. The select waves never wait on each other, so a
// sum would let a fast one cover for a slow one: each publishes its own completed-iteration count
// and the transform waves wait for all eight. A wave's LDS reads and writes complete (lgkmcnt(0))
// before its lane 0 publishes; waiters look every 64 clocks (s_sleep 1).
__device__ __forceinline__ void lds_publish_wait() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0), vmcnt / expcnt untouched
}
__device__ __forceinline__ void lds_arrive(uint32_t* c, int lane) {
    lds_publish_wait();
    if (lane == 0) __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_publish(uint32_t* c, int lane, uint32_t v) {
    lds_publish_wait();
    if (lane == 0) __hip_atomic_store(c, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_wait_ge(const uint32_t* c, uint32_t target) {
    for (;;) {
        const uint32_t v = __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if ((uint32_t)__builtin_amdgcn_readfirstlane((int)v) >= target) break;
        __builtin_amdgcn_s_sleep(MKID_F3_SLEEP);
    }
    asm volatile("" ::: "memory");
}
// every one of the 8 words c[0..7] >= target (lane l looks at c[l & 7])
__device__ __forceinline__ void lds_wait_all8_ge(const uint32_t* c, int lane, uint32_t target) {
    for (;;) {
        const uint32_t v = __hip_atomic_load(c + (lane & 7), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (__builtin_amdgcn_ballot_w64(v >= target) == ~0ull) break;
        __builtin_amdgcn_s_sleep(MKID_F3_SLEEP);
    }
    asm volatile("" ::: "memory");
}

template <int N>
struct G3 {
    static constexpr int NW = N / 512;
    static constexpr int FW = 8;                       // transform waves
    static constexpr int F = FW / NW;                  // frames per iteration
    static constexpr int BT = 1024;
    static constexpr int SPT = BT - FW * 64;           // select threads
    static constexpr int M = N / 2, C = N / 2, T = kPfbTaps;
    static constexpr int CPT = C / SPT;                // channels per select thread
    static constexpr int RS = 2 * T - 1 + 2 * F;       // ring slots (hops)
    static constexpr int REG = 576;
    static constexpr int FB = NW * REG;
    static constexpr size_t off_fbuf = (size_t)RS * M * 4;
    static constexpr int NB = MKID_F3_DECOUPLE ? 3 : 2;   // Y buffers
    static constexpr size_t off_tw1 = off_fbuf + (size_t)NB * F * FB * 8;
    static constexpr size_t off_tw2 = off_tw1 + (size_t)7 * 64 * 8;
    static constexpr size_t off_cnt = off_tw2 + (size_t)7 * 8 * 8;
    static constexpr size_t lds_bytes = off_cnt + 64;   // [0] transform arrivals, [8..15] select
    static_assert(N == 2048 && F == 2 && CPT == 2 && F * M == FW * 64 * 4, "k_front3 geometry");
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
    constexpr int NW = G::NW, M = G::M, C = G::C, T = G::T, RS = G::RS, F = G::F, CPT = G::CPT;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t* ring = reinterpret_cast<uint32_t*>(smem);
    float2* fbuf = reinterpret_cast<float2*>(smem + G::off_fbuf);
    float2* tw1 = reinterpret_cast<float2*>(smem + G::off_tw1);
    float2* tw2 = reinterpret_cast<float2*>(smem + G::off_tw2);
    [[maybe_unused]] uint32_t* cnt = reinterpret_cast<uint32_t*>(smem + G::off_cnt);

    const int tid = threadIdx.x;
    const int L = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
// k_front3's raw / phase stores: plain. With the slot order a wave's store instruction covers its
// 64 channels' positions within 2 (raw) or 4 (phase) lines in any lane order; non-temporal partial
// lines cost k_front3 +1.3 % and the trigger that reads them back +10 % (A/B
// profiles/r03_h_kbench_f3_slot_order2.json), plain ones are merged in L2
#ifndef MKID_F3_NT_STORES
#define MKID_F3_NT_STORES 0
#endif
#ifndef MKID_F3_INTERLEAVE
#define MKID_F3_INTERLEAVE 0
#endif
#if MKID_F3_INTERLEAVE
    // roles alternate by age on each SIMD (waves i, i+4, i+8, i+12 share one): transform waves
    // 0-3 and 8-11, select waves 4-7 and 12-15
    const bool xform = ((wave >> 2) & 1) == 0;
    const int rw = (wave & 3) | ((wave >> 3) << 2);   // index within its role
#else
    const bool xform = wave < G::FW;
    const int rw = xform ? wave : wave - G::FW;
#endif
    constexpr int SW = G::BT / 64 - G::FW;            // select waves
    static_assert(SW == 8, "one progress word per select wave");
    if (tid < 16) cnt[tid] = 0;                       // visible after the prologue barrier

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

#ifndef MKID_F3_PRIO_X
#define MKID_F3_PRIO_X 0
#endif
#ifndef MKID_F3_PRIO_S
#define MKID_F3_PRIO_S 0
#endif
// MKID_F3_PRIO_Y / _SY: priority of the YOUNGER transform waves (4-7) / select waves (12-15). Waves i,
// i + 4, i + 8, i + 12 share a SIMD and issue is arbitrated by age: stamps show waves 4-7 at ~3.5k
// work cycles per iteration against ~2.75k for 0-3 (select: 12-15 ~3.1k, 8-11 ~2.5k), and the barrier
// waits for the slowest
#ifndef MKID_F3_PRIO_Y
#define MKID_F3_PRIO_Y 0
#endif
#ifndef MKID_F3_PRIO_SY
#define MKID_F3_PRIO_SY 0
#endif
    if (xform) {
        // ---------------- transform waves: PFB + 512-point sub-FFT of (frame slot, w) ----------
        if (MKID_F3_PRIO_X) __builtin_amdgcn_s_setprio(MKID_F3_PRIO_X);
        if (MKID_F3_PRIO_Y && rw >= G::FW / 2) __builtin_amdgcn_s_setprio(MKID_F3_PRIO_Y);
        const int slot = rw / NW, w = rw % NW;
        const int xt = rw * 64 + L;                            // thread index among the transform waves
        const int qh = (xt * 4) / M, qoff = (xt * 4) % M;      // this thread's ring write
        {   // prologue: hops k_start-2T+1 .. k_start+F-1
            const int64_t h0 = k_start - 2 * T + 1;
            for (int g = 0; g < 2 * T - 1 + F; g += 2) {
                const int64_t hop = h0 + g + qh;
                if (hop > h0 + 2 * T - 2 + F) continue;
                const uint4 v = load4<N>(a, h0 + g, xt);
#if MKID_F3_PAIRRING
                ring3_put(ring + (int)(((hop % RS) + RS) % RS) * M, qoff, v);
#else
                ring_put<N>(ring + (int)(((hop % RS) + RS) % RS) * M, qoff, v);
#endif
            }
        }
        uint2 tq[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) tq[r] = a.pfbq[NW * (64 * r + L) + w];
        const int la = L & 7, kl = L >> 3;
        const float2* t1 = tw1 + L;
        const float2* t2 = tw2 + la;
        int rb = (int)((((k_start + 1 - 2 * T) % RS) + RS) % RS);   // slot of hop k - 2T + 1
        __syncthreads();
#if MKID_F3_TWREG
        // the lane's 14 twiddles are the same every iteration: held in VGPRs (the transform path
        // has registers to spare), 14 fewer LDS reads per sub-FFT on an LDS that is ~60 % busy
        float2 w1[7], w2[7];
#pragma unroll
        for (int k = 1; k < 8; ++k) {
            w1[k - 1] = t1[64 * (k - 1)];
            w2[k - 1] = t2[8 * (k - 1)];
            asm volatile("" : "+v"(w1[k - 1].x), "+v"(w1[k - 1].y), "+v"(w2[k - 1].x), "+v"(w2[k - 1].y));
        }
#endif
        for (int t = 0; t < nit + (MKID_F3_DECOUPLE ? 0 : 1); ++t) {
            STAMP3(0);
            if (t < nit) {
                const int kr = -kLpfHist + F * t;
                // the hops iteration t + 1 adds: loaded now, written after this wave's PFB
                const uint4 pre = load4<N>(a, k_b + kr + F, xt);
#if MKID_F3_DECOUPLE
                STAMP3(6);
                if (t > 0) lds_wait_ge(cnt, G::FW * t);             // every ring refill of t - 1 landed
                if (t >= 3) lds_wait_all8_ge(cnt + 8, L, t - 2);     // Y buffer t % 3 read by select t - 2
                STAMP3(7);
#endif
                float2* reg = fbuf + ((t % G::NB) * F + slot) * G::FB + w * G::REG;
                int sb = rb + slot;
                sb -= sb >= RS ? RS : 0;
                float2 v[8];
#if MKID_F3_PAIRRING
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
#endif
#pragma unroll
                for (int r = 0; r < 8; ++r) {
                    uint32_t x4[T];
#if MKID_F3_PAIRRING
#pragma unroll
                    for (int tau = 0; tau < T; ++tau) x4[tau] = xr[r][tau];
#else
                    const int hi = r >> 2;
                    const int pos = w * (M / NW) + 64 * (r & 3) + L;
#pragma unroll
                    for (int tau = 0; tau < T; ++tau) {
                        int sl = sb + 2 * tau + hi;
                        sl -= sl >= RS ? RS : 0;
                        x4[tau] = ring[sl * M + pos];
                    }
#endif
                    const uint32_t i01 = __builtin_amdgcn_perm(x4[1], x4[0], 0x05040100u);
                    const uint32_t q01 = __builtin_amdgcn_perm(x4[1], x4[0], 0x07060302u);
                    const uint32_t i23 = __builtin_amdgcn_perm(x4[3], x4[2], 0x05040100u);
                    const uint32_t q23 = __builtin_amdgcn_perm(x4[3], x4[2], 0x07060302u);
                    int32_t ai = dot2_first(tq[r].x, i01);
                    ai = __builtin_amdgcn_sdot2(as_s2(tq[r].y), as_s2(i23), ai, false);
                    int32_t aq = dot2_first(tq[r].x, q01);
                    aq = __builtin_amdgcn_sdot2(as_s2(tq[r].y), as_s2(q23), aq, false);
                    v[r] = make_float2((float)ai, (float)aq);
                }
                dft<8>(v);
#pragma unroll
#if MKID_F3_TWREG
                for (int k = 1; k < 8; ++k) v[k] = MKID_CMUL(v[k], w1[k - 1]);
#else
                for (int k = 1; k < 8; ++k) v[k] = MKID_CMUL(v[k], t1[64 * (k - 1)]);
#endif
#if MKID_F3_T1LDS
                t1_lds(v, reg, L);
#else
                t1_transpose(v);
#endif
                dft<8>(v);
#pragma unroll
#if MKID_F3_TWREG
                for (int k = 1; k < 8; ++k) v[k] = MKID_CMUL(v[k], w2[k - 1]);
#else
                for (int k = 1; k < 8; ++k) v[k] = MKID_CMUL(v[k], t2[8 * (k - 1)]);
#endif
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
                // ring refill: hops k+F .. k+2F-1 over hops k-2T-1 .. (no reader this iteration)
                int ws = rb + 2 * T - 1 + F + qh;
                ws -= ws >= RS ? RS : 0;
                ws -= ws >= RS ? RS : 0;
                #if MKID_F3_PAIRRING
                ring3_put(ring + ws * M, qoff, pre);
#else
                ring_put<N>(ring + ws * M, qoff, pre);
#endif
                rb += F;
                rb -= rb >= RS ? RS : 0;
            }
            STAMP3(1);
#if MKID_F3_DECOUPLE
            lds_arrive(cnt, L);
#else
            __syncthreads();
#endif
            STAMP3(2);
        }
    } else {
        // ---------------- select waves: channels st + SPT q, one iteration behind ---------------
        if (MKID_F3_PRIO_S) __builtin_amdgcn_s_setprio(MKID_F3_PRIO_S);
        if (MKID_F3_PRIO_SY && rw >= SW / 2) __builtin_amdgcn_s_setprio(MKID_F3_PRIO_SY);
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
        int lrow = (int)((a.k0 + k_start) & (int64_t)(a.P - 1));
        __syncthreads();
        for (int t = MKID_F3_DECOUPLE ? 1 : 0; t <= nit; ++t) {
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
#if MKID_F3_DECOUPLE
                STAMP3(8);
                lds_wait_ge(cnt, G::FW * t);                        // transform t - 1 wrote Y
                STAMP3(9);
#endif
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
                        z[q] = MKID_CMUL(X, lov[f][q]);
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
#if MKID_F3_NT_STORES
#ifndef MKID_XP_STAMPS
                                if (phase_run) __builtin_nontemporal_store(ph, phase_run + jr * C + c);
#endif
                                __builtin_nontemporal_store((int16_t)qv, raw_run + jr * C + c);
#else
                                if (phase_run) (phase_run + jr * C)[c] = ph;
                                (raw_run + jr * C)[c] = (int16_t)qv;
#endif
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
#if MKID_F3_DECOUPLE
            lds_publish(cnt + 8 + rw, L, (uint32_t)t);
#else
            __syncthreads();
#endif
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
#ifndef MKID_F2_BLOCKS_PER_CU
#define MKID_F2_BLOCKS_PER_CU 1
#endif
    const int64_t ncu = a.ncu > 0 ? a.ncu : 256;
    int64_t fpb = a.K / ((int64_t)MKID_F2_BLOCKS_PER_CU * ncu * (2048 / N));
    fpb = fpb < 64 ? 64 : (fpb > 4096 ? 4096 : fpb);
    fpb = (fpb + G::FPB - 1) / G::FPB * G::FPB;
    a.frames_per_block = fpb;
    const int64_t blocks = (a.K + fpb - 1) / fpb;
    hipLaunchKernelGGL(k_front2<N>, dim3((unsigned)blocks), dim3(G::BT), G::lds_bytes, s, a);
    return hipGetLastError();
}

hipError_t launch_front2(int N, const FrontArgs& a, hipStream_t s) {
    if (N == 2048 && a.variant == 3) return launch_front3_n<2048>(a, s);
    switch (N) {
        case 512: return launch_front2_n<512>(a, s);
        case 1024: return launch_front2_n<1024>(a, s);
        case 2048: return launch_front2_n<2048>(a, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace mkid
