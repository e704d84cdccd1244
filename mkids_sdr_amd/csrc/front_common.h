// Helpers shared by the fused front ends (k_front3.hip, k_front5.hip):
// the exact int16 PFB dot product, the 512-point sub-FFT's in-wave LDS transpose and Y swizzle,
// the paired ring-plane index, and the 16-byte hop loader.
#pragma once
#include "fft_common.h"
#include "mkid_internal.h"

namespace mkid {
namespace {

typedef short fshort2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ fshort2_t as_s2(uint32_t v) { return __builtin_bit_cast(fshort2_t, v); }
// v_dot2_i32_i16 with a zero accumulator: h.lo * x.lo + h.hi * x.hi, exact in int32
__device__ __forceinline__ int32_t dot2_first(uint32_t h, uint32_t x) {
    int32_t d;
    asm("v_dot2_i32_i16 %0, %1, %2, 0" : "=v"(d) : "v"(h), "v"(x));
    return d;
}

// the I (sel kPermI) or Q (kPermQ) halves of two packed I/Q words: lo16 from b, hi16 from a
constexpr uint32_t kPermI = 0x05040100u, kPermQ = 0x07060302u;

// Y_w[k] of a 512-point sub-FFT at k ^ ((k >> 2) & 14) of its region: the stage-3 writes and the
// select's bin-indexed reads are both conflict-free or near it (tools/front2_layouts.py)
__device__ __forceinline__ int yswz(int k) { return k ^ ((k >> 2) & 14); }

// Paired plane index: plane index i = 64 j + l (j = 0..3) at 128 (j >> 1) + 2 l + (j & 1), so a
// lane's PFB points j and j + 1 are one ds_read_b64 (conflict-free: 32 lanes x 2 dwords)
__device__ __forceinline__ int ring3_idx(int i) { return 128 * (i >> 7) + 2 * (i & 63) + ((i >> 6) & 1); }

// T1 through the wave's own LDS region: element (lane 8 kl + la, register r) goes to (lane 8 r + la,
// register kl). Lane L writes register r at 72 r + L; lane L' reads register r' at 72 (L' >> 3) +
// 8 r' + (L' & 7). Both patterns are bank-conflict-free for ds_*_b64 (writes: 32 consecutive
// entries; reads: entries 8 (r + r') + la mod 32 distinct over a lane group, r = L' >> 3 < 4
// there), every offset an immediate. 8 writes + 8 reads replace 32 VALU cross-lane moves (DPP
// row_ror:8 + v_permlane16/32_swap), which cost more on VALU-issue-bound transform waves
// (-3.9 % k_front3 at N = 2048, round 3: DESIGN.md §5.2).
__device__ __forceinline__ void t1_lds(float2 (&v)[8], float2* reg, int L) {
#pragma unroll
    for (int r = 0; r < 8; ++r) reg[72 * r + L] = v[r];
    __builtin_amdgcn_wave_barrier();
    const float2* rd = reg + 72 * (L >> 3) + (L & 7);
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] = rd[8 * r];
    __builtin_amdgcn_wave_barrier();
}

// 16 bytes (4 samples) at sample tid * 4 of the hops starting at first_hop (hop = M samples):
// non-temporal loads from the chunk (every ADC byte is read once), the call's history (the last
// front_hist_samples of the previous call) before it, zeros past the chunk's end
template <int M>
__device__ __forceinline__ uint4 front_load4(const FrontArgs& a, int64_t first_hop, int tid) {
    constexpr int64_t HIST = (int64_t)(2 * kPfbTaps - 1 + kLpfHist) * M;
    const int64_t s0 = first_hop * M + (int64_t)tid * 4;
    if (s0 >= a.K * M) return make_uint4(0, 0, 0, 0);
    if (s0 >= -a.avail) {
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a.x + s0));
        return make_uint4(v.x, v.y, v.z, v.w);
    }
    return *reinterpret_cast<const uint4*>(a.xhist + (s0 + a.avail + HIST));
}

// front_load4 as one unconditional load (no branch around it, so that the compiler's wait for it
// can count the loads issued after it): the address is selected, and a load past the chunk's end
// reads the chunk's first word and is zeroed by the caller where it is used (past)
struct Load4 {
    uint4 v;
    bool past;
};
template <int M>
__device__ __forceinline__ Load4 front_load4_nb(const FrontArgs& a, int64_t first_hop, int tid) {
    constexpr int64_t HIST = (int64_t)(2 * kPfbTaps - 1 + kLpfHist) * M;
    const int64_t s0 = first_hop * M + (int64_t)tid * 4;
    const bool past = s0 >= a.K * M;
    const uint32_t* p = s0 >= -a.avail ? a.x + (past ? 0 : s0) : a.xhist + (s0 + a.avail + HIST);
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return Load4{make_uint4(v.x, v.y, v.z, v.w), past};
}

}  // namespace
}  // namespace mkid
