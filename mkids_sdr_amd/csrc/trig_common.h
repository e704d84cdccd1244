// One sample of the K7/K8 trigger recurrence, shared by the serial, speculative and fix-up
// kernels. Integer semantics bit-identical to oracle/trigger.c (reference anchors listed there).
#pragma once
#include "mkid_internal.h"

namespace mkid {

enum { ST_ARMED = 0, ST_PULSE = 1, ST_DEAD = 2, ST_REARM = 3 };

struct TrigCfg {
    int32_t thr, rearm, mode, alpha, kf, kq, base_thr, dead;   // rearm: the channel's re-arm level
};

__device__ __forceinline__ int32_t tclamp16(int32_t v) { return v < -32768 ? -32768 : (v > 32767 ? 32767 : v); }
__device__ __forceinline__ int32_t tclampi(int32_t v, int32_t lo, int32_t hi) { return v < lo ? lo : (v > hi ? hi : v); }

__device__ __forceinline__ int64_t peakfit_i(int64_t y1, int64_t y2, int64_t y3) {
    const int64_t den = y3 + y1 - 2 * y2;
    if (den == 0) return y2;
    const int64_t d = y3 - y1;
    return y2 - (d * d) / (8 * den);
}

__device__ __forceinline__ uint64_t pack_wide(int32_t ch, int64_t peak, int32_t base, int64_t j) {
    const uint64_t pk = (uint64_t)tclampi((int32_t)((peak >> 4) + 2048), 0, 4095);
    const uint64_t bs = (uint64_t)tclampi((base >> 4) + 2048, 0, 4095);
    return ((uint64_t)(ch & 0xFFF) << MKID_PKT_CH_SHIFT) | (pk << MKID_PKT_PEAK_SHIFT) |
           (bs << MKID_PKT_BASE_SHIFT) | ((uint64_t)j & MKID_PKT_TS_MASK);
}

// Matched-filter output from the 26-sample window: tap i multiplies raw_{j-i}.
__device__ __forceinline__ int32_t mf_out(int32_t acc) { return tclamp16(acc >> 11); }

// What a packet needs besides the current sample: the two previous filtered samples and the
// baseline the trigger compared against.
struct EvInfo {
    int32_t y1, y2, base;
};

// Packet assembly is out of line: it runs once per event (int64 parabolic fit with a division),
// and keeping it out of the 26-fold unrolled sample loops keeps those loops small.
__device__ __attribute__((noinline)) uint64_t make_packet(int32_t c, EvInfo ev, int32_t f, int64_t jg);

// Advance state s by one filtered sample f. Returns true when a packet is due; ev then holds
// its inputs (the packet is stamped jg - 1: the peak is the previous sample).
__device__ __forceinline__ bool trig_update(TrigState& s, int32_t f, const TrigCfg& k, EvInfo& ev) {
    // the baseline starts at the first sample after the start-of-stream hold-off (a reset leaves
    // the state DEAD for kHoldOff samples with no baseline, oracle/trigger.c HOLDOFF)
    if (!s.binit && s.st != ST_DEAD) {
        s.B = (k.mode == MKID_BASE_NONE) ? 0 : f;
        s.low = (int64_t)f * 65536;
        s.band = 0;
        s.binit = 1;
    }
    const int32_t base_prev = (k.mode == MKID_BASE_SVF) ? (int32_t)(s.low >> 16) : s.B;
    const int32_t e = f - base_prev;
    const bool gate = (k.base_thr <= 0) || (e < k.base_thr && e > -k.base_thr);
    if (k.mode == MKID_BASE_EMA && s.binit) {
        s.B += gate ? ((k.alpha * e) >> 9) : 0;
    } else if (k.mode == MKID_BASE_SVF && gate && s.binit) {
        const int64_t high = ((int64_t)f * 65536) - s.low - (((int64_t)k.kq * s.band) >> 16);
        s.band += ((int64_t)k.kf * high) >> 16;
        s.low += ((int64_t)k.kf * s.band) >> 16;
    }
    // state machine as selects: lanes are channels in different states, branches would diverge
    const bool armed = s.st == ST_ARMED, pulse = s.st == ST_PULSE, dead = s.st == ST_DEAD;
    const bool rearm = s.st == ST_REARM;
    const bool emit = pulse && (f > s.f1);
    const int32_t cnt1 = s.cnt - 1;
    const bool to_pulse = armed && (e < k.thr);
    const bool to_rearm = dead && (cnt1 <= 0);
    const bool to_armed = rearm && (e >= k.rearm);   // re-arm level (hysteresis; = thr without)
    ev = EvInfo{s.f2, s.f1, base_prev};
    s.cnt = emit ? k.dead : (dead ? cnt1 : s.cnt);
    s.st = to_pulse ? ST_PULSE : (emit ? ST_DEAD : (to_rearm ? ST_REARM : (to_armed ? ST_ARMED : s.st)));
    s.f2 = s.f1;
    s.f1 = f;
    return emit;
}

// A state in the start-of-stream hold-off (DEAD, baseline not yet set) must run trig_update:
// the fast form below assumes the baseline is settled.
__device__ __forceinline__ bool in_holdoff(const TrigState& s) { return !s.binit && s.st == ST_DEAD; }

// Hot-loop form of trig_update for the EMA and no-baseline modes (k_trig_spec), same outputs:
//  * the state machine is one code x: ARMED -1, PULSE -2, REARM 0, DEAD = dead-time samples
//    left (>= 1). ARMED/REARM share one rule (x' = e < lv ? 2x : -1 with lv = thr in ARMED and the
//    re-arm level in REARM), DEAD counts down into
//    REARM, PULSE emits into DEAD max(dead, 1) (a DEAD count <= 0 behaves exactly like 1);
//  * the baseline is already initialised (binit is settled once before the loop);
//  * the dead-band gate |e| < base_thr is one unsigned compare (goff/glim), and alpha * e a
//    24-bit multiply (alpha <= 1024 keeps |e| < 2^18: exact).
struct FastState {
    int32_t B, x, f1, f2;
};
struct FastCfg {
    int32_t thr, rearm, alpha, dx;
    uint32_t goff, glim;
};

__device__ __forceinline__ FastCfg fast_cfg(const TrigCfg& k) {
    FastCfg q{k.thr, k.rearm, k.alpha, k.dead > 1 ? k.dead : 1, 0x80000000u, 0xffffffffu};
    if (k.base_thr > 0) {
        q.goff = (uint32_t)k.base_thr - 1u;
        q.glim = 2u * (uint32_t)k.base_thr - 1u;
    }
    return q;
}

__device__ __forceinline__ FastState to_fast(const TrigState& s) {
    const int32_t x = s.st == ST_ARMED ? -1 : (s.st == ST_PULSE ? -2 : (s.st == ST_REARM ? 0 : (s.cnt > 1 ? s.cnt : 1)));
    return FastState{s.B, x, s.f1, s.f2};
}

__device__ __forceinline__ TrigState from_fast(const FastState& f) {
    const int32_t st = f.x == -1 ? ST_ARMED : (f.x == -2 ? ST_PULSE : (f.x == 0 ? ST_REARM : ST_DEAD));
    return TrigState{f.B, 1, st, f.x > 0 ? f.x : 0, f.f1, f.f2, 0, 0, 0, 0};
}

template <int MODE>
__device__ __forceinline__ bool trig_update_fast(FastState& s, int32_t f, const FastCfg& k, EvInfo& ev) {
    const int32_t e = f - s.B;
    ev = EvInfo{s.f2, s.f1, s.B};
    if (MODE == MKID_BASE_EMA) {
        // branch-free: as a branch the update splits every sample into its own block, and the
        // register allocator of the unrolled 26-sample groups spills across them
        const int32_t gate = -(int32_t)((uint32_t)e + k.goff < k.glim);
        s.B += (__mul24(k.alpha, e) >> 9) & gate;
    }
    const int32_t x = s.x;
    const bool emit = (x == -2) & (f > s.f1);
    int32_t xn = e < (x == 0 ? k.rearm : k.thr) ? 2 * x : -1;
    xn = x == -2 ? (f > s.f1 ? k.dx : -2) : xn;
    xn = x > 0 ? x - 1 : xn;
    s.x = xn;
    s.f2 = s.f1;
    s.f1 = f;
    return emit;
}

// Hot-loop form of trig_update for the SVF mode (same outputs): the code-state machine of
// trig_update_fast, the Chamberlin update in int64 exactly as trig_update (floor shifts), the
// baseline settled before the loop. ev.base is low >> 16, the baseline the sample is compared to.
struct FastSvf {
    int64_t low, band;
    int32_t x, f1, f2;
};

__device__ __forceinline__ FastSvf to_fast_svf(const TrigState& s) {
    const FastState f = to_fast(s);
    return FastSvf{s.low, s.band, f.x, f.f1, f.f2};
}

__device__ __forceinline__ TrigState from_fast_svf(const FastSvf& f) {
    TrigState t = from_fast(FastState{0, f.x, f.f1, f.f2});
    t.low = f.low;
    t.band = f.band;
    return t;
}

// a * b (mod 2^64, i.e. the int64 product whenever it does not overflow) for 0 <= a < 2^32:
// v_mad_u64_u32 + v_mul_lo_u32, where the generic int64 x int64 product takes three multiplies
__device__ __forceinline__ int64_t mul_u32_i64(uint32_t a, int64_t b) {
    const uint64_t lo = (uint64_t)a * (uint32_t)b;
    const uint32_t hi = a * (uint32_t)((uint64_t)b >> 32);
    return (int64_t)(lo + ((uint64_t)hi << 32));
}

__device__ __forceinline__ void base_update_svf(FastSvf& s, int32_t f, const FastCfg& k, int32_t kf, int32_t kq) {
    const int32_t e = f - (int32_t)(s.low >> 16);
    const bool gate = (uint32_t)e + k.goff < k.glim;
    const int64_t high = ((int64_t)f * 65536) - s.low - (mul_u32_i64((uint32_t)kq, s.band) >> 16);
    const int64_t band = s.band + (mul_u32_i64((uint32_t)kf, high) >> 16);
    const int64_t low = s.low + (mul_u32_i64((uint32_t)kf, band) >> 16);
    s.band = gate ? band : s.band;
    s.low = gate ? low : s.low;
    s.f2 = s.f1;
    s.f1 = f;
}

__device__ __forceinline__ bool trig_update_svf(FastSvf& s, int32_t f, const FastCfg& k, int32_t kf, int32_t kq,
                                                EvInfo& ev) {
    const int32_t base = (int32_t)(s.low >> 16);
    const int32_t e = f - base;
    ev = EvInfo{s.f2, s.f1, base};
    {   // computed unconditionally and selected (a branch per sample splits the unrolled groups
        // into blocks the register allocator spills across)
        const bool gate = (uint32_t)e + k.goff < k.glim;
        // kf, kq are Fix18_16 in 0..2^18-1 (mkid_set_baseline checks)
        const int64_t high = ((int64_t)f * 65536) - s.low - (mul_u32_i64((uint32_t)kq, s.band) >> 16);
        const int64_t band = s.band + (mul_u32_i64((uint32_t)kf, high) >> 16);
        const int64_t low = s.low + (mul_u32_i64((uint32_t)kf, band) >> 16);
        s.band = gate ? band : s.band;
        s.low = gate ? low : s.low;
    }
    const int32_t x = s.x;
    const bool emit = (x == -2) & (f > s.f1);
    int32_t xn = e < (x == 0 ? k.rearm : k.thr) ? 2 * x : -1;
    xn = x == -2 ? (f > s.f1 ? k.dx : -2) : xn;
    xn = x > 0 ? x - 1 : xn;
    s.x = xn;
    s.f2 = s.f1;
    s.f1 = f;
    return emit;
}

// Baseline-only forms for the early part of a long speculative warm-up: the baseline (EMA B /
// SVF low, band) and the last two samples advance, the trigger state machine does not. Whatever
// state machine code results is re-converged by the full steps of the warm-up's last part and,
// like every speculated start state, verified exactly by k_trig_fix.
template <int MODE>
__device__ __forceinline__ void base_update_fast(FastState& s, int32_t f, const FastCfg& k) {
    if (MODE == MKID_BASE_EMA) {
        const int32_t e = f - s.B;
        const int32_t gate = -(int32_t)((uint32_t)e + k.goff < k.glim);
        s.B += (__mul24(k.alpha, e) >> 9) & gate;
    }
    s.f2 = s.f1;
    s.f1 = f;
}

// Advance state s by one filtered sample f taken at global phase index jg. Returns true and fills
// *pkt when a packet is emitted (its timestamp is jg - 1: the peak is the previous sample).
__device__ __forceinline__ bool trig_step(TrigState& s, int32_t f, const TrigCfg& k, int32_t c,
                                          int64_t jg, uint64_t* pkt) {
    EvInfo ev;
    if (!trig_update(s, f, k, ev)) return false;
    *pkt = make_packet(c, ev, f, jg);
    return true;
}

// Equality of the parts of the state that influence future outputs (dead-time counter only in
// ST_DEAD; B only for EMA; low/band only for SVF). Two trajectories with equal canonical state
// and equal inputs produce identical packets from then on.
// state_eq without branches, for states already in registers (k_trig_fix's check of every segment
// boundary: with the short-circuit form each lane's later fields were loaded behind a branch, a
// dependent memory round trip per field group)
__device__ __forceinline__ bool state_eq_nb(const TrigState& a, const TrigState& b, int mode) {
    bool eq = (a.binit == b.binit) & (a.st == b.st) & (a.f1 == b.f1) & (a.f2 == b.f2);
    eq &= (a.st != ST_DEAD) | (a.cnt == b.cnt);
    const bool base = mode == MKID_BASE_EMA ? a.B == b.B
                                            : (mode == MKID_BASE_SVF ? (a.low == b.low) & (a.band == b.band) : true);
    return eq & (!a.binit | base);
}

__device__ __forceinline__ bool state_eq(const TrigState& a, const TrigState& b, int mode) {
    if (a.binit != b.binit || a.st != b.st || a.f1 != b.f1 || a.f2 != b.f2) return false;
    if (a.st == ST_DEAD && a.cnt != b.cnt) return false;
    if (!a.binit) return true;
    if (mode == MKID_BASE_EMA) return a.B == b.B;
    if (mode == MKID_BASE_SVF) return a.low == b.low && a.band == b.band;
    return true;
}

}  // namespace mkid
