// Radix-2/4/8 forward DFT butterflies and Stockham LDS passes for the channeliser FFT.
// Sign convention: X[k] = sum_n x[n] exp(-2 pi i n k / N) (numpy.fft.fft).
#pragma once
#include <hip/hip_runtime.h>

namespace mkid {

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
    return make_float2(fmaf(a.x, b.x, -a.y * b.y), fmaf(a.x, b.y, a.y * b.x));
}
__device__ __forceinline__ float2 mul_mi(float2 a) { return make_float2(a.y, -a.x); }  // -i * a

// Packed-FP32 forms of the rotations by -+i: one v_pk_add_f32 whose op_sel swaps the halves of
// the second operand (the compiler otherwise materialises the swap with v_mov pairs).
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2v f2v_of(float2 a) { return f2v{a.x, a.y}; }
__device__ __forceinline__ float2 float2_of(f2v a) { return make_float2(a.x, a.y); }
// a + (-i) b = (a.x + b.y, a.y - b.x)
__device__ __forceinline__ float2 add_mi(float2 a, float2 b) {
    f2v d;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(d) : "v"(f2v_of(a)), "v"(f2v_of(b)));
    return float2_of(d);
}
// a - (-i) b = a + i b = (a.x - b.y, a.y + b.x)
__device__ __forceinline__ float2 sub_mi(float2 a, float2 b) {
    f2v d;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(d) : "v"(f2v_of(a)), "v"(f2v_of(b)));
    return float2_of(d);
}
// (a.x + a.y, a.y - a.x) = (1 - i) a   (the W8 rotations up to a real scale)
__device__ __forceinline__ float2 rot_1mi(float2 a) {
    f2v d;
    asm("v_pk_add_f32 %0, %1, %1 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(d) : "v"(f2v_of(a)));
    return float2_of(d);
}
// x + s * a for a real scalar s (one v_pk_fma_f32, s broadcast to both halves)
__device__ __forceinline__ float2 fma_s(float2 a, float s, float2 x) {
    f2v d;
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1]" : "=v"(d) : "v"(f2v_of(a)), "v"(f2v{s, s}), "v"(f2v_of(x)));
    return float2_of(d);
}
// x + t * y (complex multiply-accumulate as two v_pk_fma_f32)
__device__ __forceinline__ float2 cmac(float2 x, float2 t, float2 y) {
    f2v d;
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1]\n\t"
        "v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_lo:[1,0,0]"
        : "=&v"(d) : "v"(f2v_of(y)), "v"(f2v_of(t)), "v"(f2v_of(x)));
    return float2_of(d);
}

// y * t as one v_pk_mul_f32 + one v_pk_fma_f32 (the plain cmul above compiles to four scalar
// FP32 ops where the operands come straight from LDS)
__device__ __forceinline__ float2 cmul_pk(float2 y, float2 t) {
    f2v d;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]\n\t"
        "v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_lo:[1,0,0]"
        : "=&v"(d) : "v"(f2v_of(y)), "v"(f2v_of(t)));
    return float2_of(d);
}

// y * t + a (the DDC with the loop centre's -c' fused in: v_pk_fma_f32 in place of the
// v_pk_mul_f32 of cmul_pk, no extra instruction)
__device__ __forceinline__ float2 cmul_add_pk(float2 y, float2 t, float2 a) {
    f2v d;
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1]\n\t"
        "v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_lo:[1,0,0]"
        : "=&v"(d) : "v"(f2v_of(y)), "v"(f2v_of(t)), "v"(f2v_of(a)));
    return float2_of(d);
}

// x + g * a with g one half of a uniform (SGPR) tap pair gp = (g_lo, g_hi): one v_pk_fma_f32
// whose op_sel / op_sel_hi pick the same half of the pair for both lanes, so 13 pairs of
// consecutive low-pass taps serve all 26 taps without duplicating any in SGPRs (the compiler
// duplicates taps per pair and runs out of SGPRs, falling back to scalar v_fmac pairs)
template <int HI>
__device__ __forceinline__ float2 fma_tap(uint64_t gp, float2 a, float2 x) {
    f2v d;
    if constexpr (HI)
        asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,1,1]" : "=v"(d) : "s"(gp), "v"(f2v_of(a)), "v"(f2v_of(x)));
    else
        asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,0,0] op_sel_hi:[0,1,1]" : "=v"(d) : "s"(gp), "v"(f2v_of(a)), "v"(f2v_of(x)));
    return float2_of(d);
}
__device__ __forceinline__ uint64_t tap_pair(float lo, float hi) {
    return (uint64_t)__builtin_bit_cast(uint32_t, lo) | ((uint64_t)__builtin_bit_cast(uint32_t, hi) << 32);
}

__device__ __forceinline__ void dft2(float2& a, float2& b) {
    float2 t = a;
    a = cadd(t, b);
    b = csub(t, b);
}

__device__ __forceinline__ void dft4(float2& v0, float2& v1, float2& v2, float2& v3) {
    const float2 s02 = cadd(v0, v2), d02 = csub(v0, v2);
    const float2 s13 = cadd(v1, v3), t13 = csub(v1, v3);
    v0 = cadd(s02, s13);
    v2 = csub(s02, s13);
    v1 = add_mi(d02, t13);  // d02 + (-i) t13
    v3 = sub_mi(d02, t13);
}

template <int R>
__device__ __forceinline__ void dft(float2* v);

template <>
__device__ __forceinline__ void dft<2>(float2* v) { dft2(v[0], v[1]); }

template <>
__device__ __forceinline__ void dft<4>(float2* v) { dft4(v[0], v[1], v[2], v[3]); }

template <>
__device__ __forceinline__ void dft<8>(float2* v) {
    constexpr float r2 = 0.70710678118654752440f;
    float2 e0 = v[0], e1 = v[2], e2 = v[4], e3 = v[6];
    float2 o0 = v[1], o1 = v[3], o2 = v[5], o3 = v[7];
    dft4(e0, e1, e2, e3);
    dft4(o0, o1, o2, o3);
    // W8^1 o1 = r2 (1 - i) o1;  W8^2 o2 = -i o2;  W8^3 o3 = -i r2 (1 - i) o3
    const float2 p1 = rot_1mi(o1);
    const float2 p3 = make_float2(rot_1mi(o3).x * r2, rot_1mi(o3).y * r2);
    v[0] = cadd(e0, o0); v[4] = csub(e0, o0);
    v[1] = fma_s(p1, r2, e1); v[5] = fma_s(p1, -r2, e1);
    v[2] = add_mi(e2, o2); v[6] = sub_mi(e2, o2);
    v[3] = add_mi(e3, p3); v[7] = sub_mi(e3, p3);
}

// LDS index padding: one float2 of pad every 16 entries (breaks power-of-two lane strides).
__device__ __forceinline__ int lpad(int i) { return i + (i >> 4); }
template <int N>
constexpr int lds_frame_elems() { return N + N / 16; }

// atan2 for the phase stage: octant reduction + degree-7 minimax polynomial in t^2 (t = min/max,
// v_rcp_f32). Max error 3.1e-7 rad (float32 output rounding near pi is 1.9e-7), Fix16_13
// rounding flips vs a float64 atan2 7.1e-4 per sample, the same as libm's float atan2f (6.7e-4);
// about 20 VALU instructions instead of ~45 for the library call. Fit: tools/atan_fit.py.
__device__ __forceinline__ float phase_atan2(float y, float x) {
    const float ax = fabsf(x), ay = fabsf(y);
    const float mx = fmaxf(ax, ay), mn = fminf(ax, ay);
    const float t = mx > 0.f ? mn * __builtin_amdgcn_rcpf(mx) : 0.f;
    const float u = t * t;
    float p = -0.00405451f;
    p = fmaf(p, u, 0.02186273f);
    p = fmaf(p, u, -0.05591200f);
    p = fmaf(p, u, 0.09642173f);
    p = fmaf(p, u, -0.13908620f);
    p = fmaf(p, u, 0.19946563f);
    p = fmaf(p, u, -0.33329860f);
    p = fmaf(p, u, 0.99999934f);
    float r = p * t;
    r = ay > ax ? 1.57079632679489662f - r : r;
    r = x < 0.f ? 3.14159265358979324f - r : r;
    return copysignf(r, y);
}

// LDS layouts of an exchange buffer: float2 index i lives at i + (i >> SH) * MUL. Pad16 (one pad
// per 16) is the default; other exchanges pick the layout that makes both their write and their
// read pattern bank-conflict-free (tools/lds_layouts.py checks candidates against the gfx950
// ds_read_b64 / ds_write_b64 banking of MI355X_MICROARCH.md §LDS).
template <int SH, int MUL>
struct LPad {
    __device__ __forceinline__ static constexpr int f(int i) { return i + (i >> SH) * MUL; }
    static constexpr int size(int n) { return n + ((n - 1) >> SH) * MUL + 1; }
};
using Pad16 = LPad<4, 1>;

// Stockham pass pieces; thread t of NT = N/PTS threads holds PTS points = PTS/R butterflies.
// Every LDS address is one per-thread base + a compile-time offset: the layouts are linear over
// the offsets each pass adds (multiples of 2^SH for reads; r NS for writes, checked per plan by
// tools/lds_layouts.py), so the compiler keeps one address VGPR per butterfly, not per point.
template <int N, int PTS, int R, typename PAD = Pad16>
__device__ __forceinline__ void st_read(const float2* buf, float2 (&v)[PTS], int t) {
    constexpr int NT = N / PTS, NB = PTS / R, NR = N / R;
    const float2* b = buf + PAD::f(t);
#pragma unroll
    for (int q = 0; q < NB; ++q)
#pragma unroll
        for (int r = 0; r < R; ++r) v[q * R + r] = b[PAD::f(q * NT + r * NR)];
}

template <int N, int PTS, int R, int NS, typename PAD = Pad16>
__device__ __forceinline__ void st_write(float2* buf, const float2 (&v)[PTS], int t) {
    constexpr int NT = N / PTS, NB = PTS / R;
#pragma unroll
    for (int q = 0; q < NB; ++q) {
        const int j = t + q * NT;
        float2* b = buf + PAD::f((j / NS) * NS * R + (j % NS));
#pragma unroll
        for (int r = 0; r < R; ++r) b[PAD::f(r * NS)] = v[q * R + r];
    }
}

template <int PTS, int R>
__device__ __forceinline__ void st_dft(float2 (&v)[PTS]) {
#pragma unroll
    for (int q = 0; q < PTS / R; ++q) dft<R>(&v[q * R]);
}

// Register-lean twiddles: one base w = exp(-2 pi i (j%NS) / (NS R)) per butterfly; the powers
// w^2..w^(R-1) are rebuilt by at most 6 complex multiplies per radix-8 butterfly (error a few ulp,
// far below the 1e-5 rad phase bar) instead of holding R-1 complex values in VGPRs.
template <int N, int PTS, int R, int NS>
struct TwiddleRec {
    static constexpr int NB = PTS / R;
    float2 w[NB];
    __device__ __forceinline__ void init(int t) {
        constexpr int NT = N / PTS;
#pragma unroll
        for (int q = 0; q < NB; ++q) {
            const int m = (t + q * NT) % NS;
            double s, c;
            sincospi(-2.0 * (double)m / (double)(NS * R), &s, &c);
            w[q] = make_float2((float)c, (float)s);
        }
    }
    __device__ __forceinline__ void apply(float2 (&v)[PTS]) const {
#pragma unroll
        for (int q = 0; q < NB; ++q) {
            float2* b = &v[q * R];
            float2 w1 = w[q];
            // opaque to the optimiser: otherwise loop-invariant code motion hoists the powers
            // out of the frame loop and they occupy registers again
            asm volatile("" : "+v"(w1.x), "+v"(w1.y));
            if constexpr (R == 2) {
                b[1] = cmul(b[1], w1);
            } else if constexpr (R == 4) {
                const float2 w2 = cmul(w1, w1);
                b[1] = cmul(b[1], w1);
                b[2] = cmul(b[2], w2);
                b[3] = cmul(b[3], cmul(w2, w1));
            } else {
                static_assert(R == 8, "radix");
                const float2 w2 = cmul(w1, w1), w4 = cmul(w2, w2), w3 = cmul(w2, w1);
                b[1] = cmul(b[1], w1);
                b[2] = cmul(b[2], w2);
                b[3] = cmul(b[3], w3);
                b[4] = cmul(b[4], w4);
                b[5] = cmul(b[5], cmul(w4, w1));
                b[6] = cmul(b[6], cmul(w4, w2));
                b[7] = cmul(b[7], cmul(w4, w3));
            }
        }
    }
};

// Twiddles of one pass read from an LDS table: w^r, w = exp(-2 pi i m / (NS R)), m = j mod NS,
// stored plane by plane (entry (r, m) at (r - 1) NS + m, 8 B each), so consecutive m are
// consecutive float2: conflict-free ds_read_b64 (2 LDS cycles each; broadcast for NS < 64)
// instead of being rebuilt by complex multiplies.
template <int N, int PTS, int R, int NS>
struct TwiddleLds {
    static constexpr int NB = PTS / R;
    static constexpr int ENTRIES = NS * (R - 1);  // float2 in the table
    const float2* tab;
    __device__ __forceinline__ static void fill(float2* tab, int tid, int nthreads) {
        for (int i = tid; i < ENTRIES; i += nthreads) {
            const int r = i / NS + 1, m = i % NS;
            double sn, cs;
            sincospi(-2.0 * (double)(m * r) / (double)(NS * R), &sn, &cs);
            tab[i] = make_float2((float)cs, (float)sn);
        }
    }
    __device__ __forceinline__ void apply(float2 (&v)[PTS], int t) const {
        constexpr int NT = N / PTS;
#pragma unroll
        for (int q = 0; q < NB; ++q) {
            const float2* e = tab + (t + q * NT) % NS;
#pragma unroll
            for (int r = 1; r < R; ++r)
                v[q * R + r] = cmul(v[q * R + r], *static_cast<const float2*>(__builtin_assume_aligned(e + (r - 1) * NS, 8)));
        }
    }
};

template <int N>
struct Plan8;  // PTS = 8 points per thread; radix sequence R1..R4 (1 = no pass)
template <> struct Plan8<128>  { static constexpr int NP = 3, R[4] = {8, 4, 4, 1}; };
template <> struct Plan8<256>  { static constexpr int NP = 3, R[4] = {8, 8, 4, 1}; };
template <> struct Plan8<512>  { static constexpr int NP = 3, R[4] = {8, 8, 8, 1}; };
template <> struct Plan8<1024> { static constexpr int NP = 4, R[4] = {8, 8, 4, 4}; };
template <> struct Plan8<2048> { static constexpr int NP = 4, R[4] = {8, 8, 8, 4}; };
template <> struct Plan8<4096> { static constexpr int NP = 4, R[4] = {8, 8, 8, 8}; };

}  // namespace mkid
