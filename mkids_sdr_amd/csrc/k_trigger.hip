// K7-K8: matched filter + baseline (EMA / SVF) + threshold + parabolic peak + dead time +
// packetiser, evaluated EXACTLY but in parallel over time by speculative segments:
//
//   k_trig_spec  thread = (channel c, segment s of L phase samples). Segment 0 starts from the
//                channel's carried state (exact). Segment s>0 starts W samples early from a guessed
//                state (re-arm pending, baseline = first filtered sample), runs the warm-up
//                silently, records its state S_spec at the segment start, then emits packets.
//   k_trig_fix   one wave per channel. Segment s is exact iff the true state at its start equals
//                S_spec[s]; by induction from the exact segment 0 that is S_end[s-1] == S_spec[s],
//                checked for all segments at once (64 per ballot). Only the failures walk
//                serially: the true and the speculative trajectories are re-run side by side from
//                the segment start until they coincide (the recurrence is deterministic in
//                (state, input)) and the packet lists are spliced: true packets before the merge,
//                speculative ones after it. A re-run that never merges hands its end state to an
//                explicit check of the next segment.
//
// The result is bit-identical to the sequential oracle/trigger.c for every input; the speculation
// only decides how much sequential work the fix-up does (EMA merges within ~10^2 samples on noisy
// phase; the slow SVF baseline needs ~10^4, so its segments warm up over kSvfW, mkid_api.hip).
// The 26-tap matched filter is 13 v_dot2_i32_i16 per sample in the walk (24-bit multiply-adds in
// the fix-up's serial re-run). In SVF mode a pre-pass (k_mf_rows) writes the filtered rows once
// and the walk reads them: its ~10^5-sample warm-up is bound by one wave's instruction stream,
// and the filter was 16 of its 40 VALU per sample.
#include <algorithm>
#include <type_traits>

#include "trig_common.h"

namespace mkid {

constexpr int kSpecThreads = 256;
// full trigger steps at the end of a speculative warm-up (groups of 26 samples): the state machine
// forgets a guessed start within the dead time plus one threshold crossing; earlier warm-up
// samples advance only the baseline (the SVF warm-up is ~10^5 samples, the EMA one 260)
constexpr int32_t kFullWarm = 100;

// Per-segment states (s_spec, s_end) channel-major, [c][s]: k_trig_fix's wave of channel c reads its
// segment boundaries as consecutive entries (one coalesced load per 64 boundaries); k_trig_spec
// writes each thread's two states once
__device__ __forceinline__ int64_t seg_state(const TrigSpecArgs& a, int c, int s) { return (int64_t)c * a.nseg + s; }

__device__ __attribute__((noinline)) uint64_t make_packet(int32_t c, EvInfo ev, int32_t f, int64_t jg) {
    return pack_wide(c, peakfit_i(ev.y1, ev.y2, f), ev.base, jg - 1);
}

struct Win {
    int32_t w[kFirTaps];
};

// Load raw_{j-25..j-1} into ring slots (j' - j + 26) % 26 of a ring aligned at j.
__device__ __forceinline__ void load_window(Win& win, const TrigSpecArgs& a, int c, int64_t j) {
    win.w[0] = 0;
#pragma unroll
    for (int i = 1; i < kFirTaps; ++i) {
        const int64_t jj = j - kFirTaps + i;  // slot i holds raw_{j-26+i}
        win.w[i] = jj >= 0 ? a.raw[jj * a.C + c]
                           : (jj >= -kRawHist ? a.rhist[(jj + kRawHist) * a.C + c] : 0);
    }
}

// filtered sample for ring position u (raw_j already stored in slot u)
__device__ __forceinline__ int32_t mf_at(const Win& win, const int32_t (&tap)[kFirTaps], int u) {
    int32_t acc = 0;
#pragma unroll
    for (int i = 0; i < kFirTaps; ++i) acc = __mul24(tap[i], win.w[(u - i + kFirTaps) % kFirTaps]) + acc;
    return mf_out(acc);
}

// Matched filter on packed pairs: q_j = (raw_j, raw_{j-1}) as two int16 in one dword, and
// tap pairs (a_2m, a_2m+1); f_j = sum_m dot2(tappair_m, q_{j-2m}) -> 13 v_dot2c_i32_i16 per sample.
typedef short short2_t __attribute__((ext_vector_type(2)));
struct QWin {
    uint32_t q[kFirTaps];  // slot (i - base) % 26 holds q_i
    uint32_t last;         // the dword holding raw_{i-1} (in the lane's half) for the next pack
    uint32_t sel;          // v_perm selector: (raw_j, raw_{j-1}) from the lane's half of two dwords
};

__device__ __forceinline__ uint32_t pack2(int32_t lo, int32_t hi) {
    return ((uint32_t)lo & 0xffffu) | ((uint32_t)hi << 16);
}

__device__ __forceinline__ short2_t as_s2(uint32_t v) { return __builtin_bit_cast(short2_t, v); }

// ring aligned at j: slots 2..25 hold q_{j-24..j-1} (slot (i - j + 26) % 26); last = raw_{j-1}
__device__ __forceinline__ void load_qwin(QWin& w, const TrigSpecArgs& a, int c, int64_t j) {
    int32_t prev = 0;
#pragma unroll
    for (int i = 0; i < kFirTaps; ++i) {
        const int64_t jj = j - kFirTaps + i;  // raw_{j-26+i}
        const int32_t r = jj >= 0 ? a.raw[jj * a.C + c]
                                  : (jj >= -kRawHist ? a.rhist[(jj + kRawHist) * a.C + c] : 0);
        w.q[i] = pack2(r, prev);
        prev = r;
    }
    w.last = pack2(prev, prev);   // raw_{j-1} in both halves: valid for either lane parity
    w.sel = (c & 1) ? 0x07060302u : 0x05040100u;
}

// r: the aligned dword holding raw_j (lanes 2k and 2k+1 load the same dword and keep their own
// half): the pack is one v_perm, and the loaded values stay 32-bit through the pipelined loop
// lim: -32768 and 32767 in VGPRs (made opaque by the caller), so that the clamp of mf_out is one
// v_med3_i32 (gfx9 VOP3 takes no literal operand; with literals it is a v_max + v_min pair)
struct Lim16 {
    int32_t lo, hi;
};
__device__ __forceinline__ int32_t mf_q(QWin& w, const uint32_t (&tp)[kFirTaps / 2], int u, uint32_t r,
                                        const Lim16& lim) {
    w.q[u] = __builtin_amdgcn_perm(w.last, r, w.sel);
    w.last = r;
    // first product into a zero accumulator (v_dot2_i32_i16 ..., 0): the compiler otherwise zeroes
    // a register for a v_dot2c chain, one extra VALU per sample
    int32_t acc;
    asm("v_dot2_i32_i16 %0, %1, %2, 0" : "=v"(acc) : "v"(tp[0]), "v"(w.q[u]));
#pragma unroll
    for (int m = 1; m < kFirTaps / 2; ++m)
        acc = __builtin_amdgcn_sdot2(as_s2(tp[m]), as_s2(w.q[(u - 2 * m + 2 * kFirTaps) % kFirTaps]), acc, false);
    int32_t v;   // mf_out: clamp16(acc >> 11)
    asm("v_med3_i32 %0, %1, %2, %3" : "=v"(v) : "v"(acc >> 11), "v"(lim.lo), "v"(lim.hi));
    return v;
}

// Buffer loads of the raw phase: the row offset rrow is wave-uniform (the instruction's SGPR offset,
// no VALU address arithmetic per load), lane the lane's constant byte offset. The descriptor
// spans 4 GiB from the wave's segment base (word 3 as ck_tile's gfx9 buffer resource).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t raw_rsrc(const char* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base), (short)0, (int)0xffffffff, 0x00020000);
}

// Software pipeline over half groups of 13 samples: the loads of the next half are in flight
// while the current half is processed (26 load registers, as for a whole-group batch, but no
// wave waits a full memory latency per group). A whole group in flight ahead (52 registers, 2 waves
// per SIMD) is +16 % at config 3 and flat at config 2 (profiles/r04/r04_l_kbench_trig_deep_c*.json).
// body(group, u, raw) sees u = 0..25 in order and half_end(group, h) runs after each half group
// (h = 0, 1); rrow advances by ngroups rows of 26. The last prefetch re-reads the current group.
template <class F, class E>
__device__ __forceinline__ void run_groups(int32_t ngroups, const char* rbase, uint32_t& rrow, uint32_t lane,
                                           uint32_t row, F&& body, E&& half_end) {
    constexpr int H = kFirTaps / 2;
    const __amdgpu_buffer_rsrc_t rs = raw_rsrc(rbase);
    auto ld = [&](uint32_t off) { return (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, (int)lane, (int)off, 0); };
    // the row offsets are wave-uniform by construction; one readfirstlane per half group says so
    // to the compiler, which otherwise may keep them in VGPRs (a VALU add + readfirstlane per load,
    // or, in the SVF warm-up, a waterfall loop around every load)
    auto uni = [](uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); };
    uint32_t ra[H], rb[H];
    if (ngroups <= 0) return;
    rrow = uni(rrow);
#pragma unroll
    for (int u = 0; u < H; ++u) ra[u] = ld(rrow + (uint32_t)u * row);
    for (int32_t g = 0; g < ngroups; ++g) {
        const uint32_t cur = uni(rrow);
#pragma unroll
        for (int u = 0; u < H; ++u) rb[u] = ld(cur + (uint32_t)(H + u) * row);
#pragma unroll
        for (int u = 0; u < H; ++u) body(g, u, ra[u]);
        half_end(g, 0);
        const uint32_t nxt = uni(cur + (g + 1 < ngroups ? (uint32_t)kFirTaps * row : 0u));
#pragma unroll
        for (int u = 0; u < H; ++u) ra[u] = ld(nxt + (uint32_t)u * row);
#pragma unroll
        for (int u = 0; u < H; ++u) body(g, H + u, rb[u]);
        half_end(g, 1);
        rrow = cur + (uint32_t)kFirTaps * row;
    }
}
template <class F>
__device__ __forceinline__ void run_groups(int32_t ngroups, const char* rbase, uint32_t& rrow, uint32_t lane,
                                           uint32_t row, F&& body) {
    run_groups(ngroups, rbase, rrow, lane, row, body, [](int32_t, int) {});
}


// The per-sample recurrence of k_trig_spec: the code-state forms trig_update_fast (EMA / no
// baseline) and trig_update_svf (SVF) on the throughput path, trig_update itself (FAST = false)
// for a segment that starts in the start-of-stream hold-off.
template <int MODE, bool FAST = true>
struct Stepper {
    TrigState st;
    TrigCfg k;
    __device__ Stepper(const TrigState& s, const TrigCfg& kk, int32_t) : st(s), k(kk) {}
    __device__ __forceinline__ bool step(int32_t f, EvInfo& ev) { return trig_update(st, f, k, ev); }
    __device__ __forceinline__ void step_base(int32_t f) {
        EvInfo ev;
        (void)trig_update(st, f, k, ev);
    }
    __device__ __forceinline__ TrigState state() const { return st; }
};

template <int MODE>
struct Stepper<MODE, true> {
    FastState fs;
    FastCfg q;
    // f0: the filtered value of the first sample, which initialises the baseline when the
    // incoming state has none yet (exactly what trig_update's binit branch does on that sample)
    __device__ Stepper(const TrigState& s, const TrigCfg& k, int32_t f0) : fs(to_fast(s)), q(fast_cfg(k)) {
        if (!s.binit) fs.B = MODE == MKID_BASE_NONE ? 0 : f0;
    }
    __device__ __forceinline__ bool step(int32_t f, EvInfo& ev) { return trig_update_fast<MODE>(fs, f, q, ev); }
    __device__ __forceinline__ void step_base(int32_t f) { base_update_fast<MODE>(fs, f, q); }
    __device__ __forceinline__ TrigState state() const { return from_fast(fs); }
};

template <>
struct Stepper<MKID_BASE_SVF, true> {
    FastSvf fs;
    FastCfg q;
    int32_t kf, kq;
    __device__ Stepper(const TrigState& s, const TrigCfg& k, int32_t f0)
        : fs(to_fast_svf(s)), q(fast_cfg(k)), kf(k.kf), kq(k.kq) {
        if (!s.binit) {   // trig_update's baseline initialisation on the first sample
            fs.low = (int64_t)f0 * 65536;
            fs.band = 0;
        }
    }
    __device__ __forceinline__ bool step(int32_t f, EvInfo& ev) { return trig_update_svf(fs, f, q, kf, kq, ev); }
    __device__ __forceinline__ void step_base(int32_t f) { base_update_svf(fs, f, q, kf, kq); }
    __device__ __forceinline__ TrigState state() const { return from_fast_svf(fs); }
};

// 4 waves per SIMD (128 VGPRs; the occupancy also sizes the segments, mkid_plan.cpp): -4.4 %
// k_trig_spec at 1024 channels and -5.4 % at 2048 against 3 waves (135 VGPRs), neutral at 256
// (profiles/r04/r04_ag_kbench_*.json); the few spilled dwords are outside the sample loops
#ifndef MKID_TRIG_MINW
#define MKID_TRIG_MINW 4
#endif
// Issue priority falls with the wave's progress through its segment (done of ng groups): the
// SIMD's older waves otherwise win every arbitration, finish first and leave the youngest to run
// alone at a lone wave's issue rate. Priority 3 -> 2 -> 1 -> 0 at 70 / 85 / 95 % is -9 % k_trig_spec
// at 1024 and 2048 channels, neutral at 256 (profiles/r04/r04_p_*, r04_q_*).
__device__ __forceinline__ void set_progress_prio(int32_t done, int32_t ng) {
    const int32_t pc = done * 100;
    if (pc >= 95 * ng) __builtin_amdgcn_s_setprio(0);
    else if (pc >= 85 * ng) __builtin_amdgcn_s_setprio(1);
    else if (pc >= 70 * ng) __builtin_amdgcn_s_setprio(2);
}

// PRE: the rows hold the matched-filter output (a.filt, k_mf_rows) instead of the raw phase: the
// walk takes f from the lane's half of the loaded dword (SVF mode, whose walk is bound by one
// wave's instruction stream over a ~10^5-sample warm-up)
template <int MODE, bool PRE = false>
__global__ __launch_bounds__(kSpecThreads, MKID_TRIG_MINW) void k_trig_spec(TrigSpecArgs a) {
    __builtin_amdgcn_s_setprio(3);
    const int64_t g = (int64_t)blockIdx.x * kSpecThreads + threadIdx.x;
    if (g >= (int64_t)a.C * a.nseg) return;
    const int C = a.C;
    const int c = (int)(g % C);  // lanes of a wave = consecutive channels (coalesced raw loads)
    const int s = (int)(g / C);
    uint32_t tp[kFirTaps / 2];
    if constexpr (!PRE) {
#pragma unroll
        for (int m = 0; m < kFirTaps / 2; ++m)
            tp[m] = pack2(a.fir[c * kFirTaps + 2 * m], a.fir[c * kFirTaps + 2 * m + 1]);
    }
    const TrigCfg k{a.thr[c], a.rearm[c], MODE, a.alpha, a.kf, a.kq, a.base_thr, a.dead};
    const int64_t seg0 = (int64_t)s * a.L;
    const int64_t seg1 = seg0 + a.L < a.J ? seg0 + a.L : a.J;
    // a segment closer than W to the sub-chunk start warms up from row 0 with the carried state
    // (exact); L and W are multiples of 26 whenever W > 0, so seg0 - jw is too
    const int64_t jw = (s == 0 || seg0 <= a.W) ? 0 : seg0 - a.W;
    QWin win;
    if constexpr (!PRE) load_qwin(win, a, c, jw);
    const int64_t sc = (int64_t)c * a.seg_stride + a.seg_off + s;
    uint64_t* slot = a.slots + sc * a.capseg;
    int32_t n = 0;
    // all lanes of a wave share the segment (64 | C): a scalar row base and a 32-bit per-lane
    // offset give SGPR-base loads (no 64-bit address arithmetic per sample)
    const char* rbase = reinterpret_cast<const char*>((PRE ? a.filt : a.raw) +
                                                      (int64_t)__builtin_amdgcn_readfirstlane((int32_t)jw) * C);
    const uint32_t lane = (uint32_t)(c >> 1) * 4u;  // byte offset of the lane's dword (C even)
    uint32_t rrow = 0;                              // wave-uniform byte offset of the current row
    const __amdgpu_buffer_rsrc_t rs = raw_rsrc(rbase);
    auto rload = [&](uint32_t off) {
        return (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, (int)lane, __builtin_amdgcn_readfirstlane((int)off), 0);
    };
    Lim16 lim{-32768, 32767};
    asm volatile("" : "+v"(lim.lo), "+v"(lim.hi));
    const uint32_t half = (uint32_t)(c & 1) * 16u;   // PRE: the lane's int16 in the loaded dword
    // filtered sample at ring position u from the loaded dword r
    auto filt = [&](QWin& w, int u, uint32_t r) -> int32_t {
        if constexpr (PRE) return __builtin_amdgcn_sbfe((int32_t)r, half, 16);
        else return mf_q(w, tp, u, r, lim);
    };
    QWin w0 = win;
    const int32_t f0 = filt(w0, 0, rload(0));
    const TrigState st0 = jw == 0 ? a.st_in[c] : TrigState{0, 0, ST_REARM, 0, 0, 0, 0, 0, 0, 0};
    auto body = [&](auto& sp) {
        // warm-up: W is a multiple of 26 (host-checked), so the ring stays aligned at seg0. A long
        // speculative warm-up (SVF) advances only the baseline until its last kFullWarm groups
        const int32_t wg = __builtin_amdgcn_readfirstlane((int32_t)(seg0 - jw) / kFirTaps);
        int32_t wbase = 0;
        if constexpr (MODE == MKID_BASE_SVF && std::is_same<std::decay_t<decltype(sp)>, Stepper<MODE, true>>::value) {
            wbase = (jw > 0 && wg > kFullWarm) ? wg - kFullWarm : 0;
            run_groups(wbase, rbase, rrow, lane, (uint32_t)(2 * C),
                       [&](int32_t, int u, uint32_t r) { sp.step_base(filt(win, u, r)); });
        }
        run_groups(wg - wbase, rbase, rrow, lane, (uint32_t)(2 * C),
                   [&](int32_t, int u, uint32_t r) {
                       EvInfo ev;
                       (void)sp.step(filt(win, u, r), ev);
                   });
        if (s > 0) a.s_spec[seg_state(a, c, s)] = sp.state();
        const int32_t len = (int32_t)(seg1 - seg0);
        const int32_t full = len - len % kFirTaps;
        const int32_t ng = __builtin_amdgcn_readfirstlane(full / kFirTaps);
        run_groups(ng, rbase, rrow, lane, (uint32_t)(2 * C),
                   [&](int32_t gr, int u, uint32_t r) {
                       const int32_t f = filt(win, u, r);
                       EvInfo ev;
                       if (sp.step(f, ev)) {
                           if (n < a.capseg) slot[n] = make_packet(c, ev, f, a.j0 + seg0 + gr * kFirTaps + u);
                           ++n;
                       }
                   },
                   [&](int32_t gr, int h) {
                       if (h == 1) set_progress_prio(gr + 1, ng);
                   });
        const int32_t gi = full;
        const int32_t left = len - gi;  // tail < 26 samples, predicated
#pragma unroll
        for (int u = 0; u < kFirTaps; ++u) {
            if (u < left) {
                const int32_t f = filt(win, u, rload(rrow + (uint32_t)(2 * u * C)));
                EvInfo ev;
                if (sp.step(f, ev)) {
                    if (n < a.capseg) slot[n] = make_packet(c, ev, f, a.j0 + seg0 + gi + u);
                    ++n;
                }
            }
        }
        a.s_end[seg_state(a, c, s)] = sp.state();
    };
    if (in_holdoff(st0)) {  // first segment after a reset: the generic recurrence
        Stepper<MODE, false> sp(st0, k, f0);
        body(sp);
    } else {
        Stepper<MODE> sp(st0, k, f0);
        body(sp);
    }
    a.counts[sc] = n;
}

// Matched-filter pre-pass of the SVF path: f_j for rows [0, J) of every channel into a.filt
// ([J][C] int16, the same Fix16_13 clamp as the walk's mf_q). Thread = (channel, block of
// rows_per rows, a multiple of 26); the block's 25-row window is loaded first (raw history
// before row 0, as in the walk). Loads and stores are buffer ops with wave-uniform row offsets.
__global__ __launch_bounds__(kSpecThreads) void k_mf_rows(TrigSpecArgs a, int32_t rows_per) {
    const int C = a.C;
    const int64_t g = (int64_t)blockIdx.x * kSpecThreads + threadIdx.x;
    const int c = (int)(g % C);
    const int64_t j0 = (g / C) * (int64_t)rows_per;
    if (j0 >= a.J) return;
    const int64_t j1 = j0 + rows_per < a.J ? j0 + rows_per : a.J;
    uint32_t tp[kFirTaps / 2];
#pragma unroll
    for (int m = 0; m < kFirTaps / 2; ++m) tp[m] = pack2(a.fir[c * kFirTaps + 2 * m], a.fir[c * kFirTaps + 2 * m + 1]);
    QWin win;
    load_qwin(win, a, c, j0);
    const int64_t jr = __builtin_amdgcn_readfirstlane((int32_t)j0);
    const char* rbase = reinterpret_cast<const char*>(a.raw + jr * C);
    const __amdgpu_buffer_rsrc_t out = raw_rsrc(reinterpret_cast<const char*>(a.filt + jr * C));
    const uint32_t lane = (uint32_t)(c >> 1) * 4u;
    const uint32_t lane16 = (uint32_t)c * 2u;
    const uint32_t row = (uint32_t)(2 * C);
    Lim16 lim{-32768, 32767};
    asm volatile("" : "+v"(lim.lo), "+v"(lim.hi));
    auto put = [&](uint32_t roff, int32_t f) {
        __builtin_amdgcn_raw_buffer_store_b16((unsigned short)f, out, (int)lane16,
                                              __builtin_amdgcn_readfirstlane((int)roff), 0);
    };
    uint32_t rrow = 0;
    const int32_t len = (int32_t)(j1 - j0);
    const int32_t ng = __builtin_amdgcn_readfirstlane(len / kFirTaps);
    run_groups(ng, rbase, rrow, lane, row, [&](int32_t gr, int u, uint32_t r) {
        put((uint32_t)(gr * kFirTaps + u) * row, mf_q(win, tp, u, r, lim));
    });
    const int32_t left = len - ng * kFirTaps;   // tail < 26 rows (last block only), predicated
    const __amdgpu_buffer_rsrc_t rs = raw_rsrc(rbase);
#pragma unroll
    for (int u = 0; u < kFirTaps; ++u) {
        if (u < left) {
            const uint32_t ro = rrow + (uint32_t)u * row;
            const uint32_t r = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, (int)lane,
                                                                            __builtin_amdgcn_readfirstlane((int)ro), 0);
            put(ro, mf_q(win, tp, u, r, lim));
        }
    }
}

// The splice of a re-run segment s of channel c into its packet slot: nt true packets (in the
// channel's scratch) up to the merge detection, then the speculative packets after the ndrop the
// speculative trajectory emitted before it. Packets both trajectories emit between the merge and
// its detection count in nt and ndrop alike, so a late detection splices the same list.
__device__ void splice_segment(const TrigSpecArgs& a, int c, int s, int32_t nt, int32_t ndrop, bool merged,
                               const uint64_t* scratch) {
    const int64_t sc = (int64_t)c * a.seg_stride + a.seg_off + s;
    uint64_t* slot = a.slots + sc * a.capseg;
    const int32_t cnt = a.counts[sc] < a.capseg ? a.counts[sc] : a.capseg;
    int32_t total = nt;
    if (merged) {
        const int32_t keep = cnt - ndrop;
        if (nt < ndrop) {
            for (int32_t i = 0; i < keep; ++i) slot[nt + i] = slot[ndrop + i];
        } else if (nt > ndrop) {
            for (int32_t i = keep - 1; i >= 0; --i)
                if (nt + i < a.capseg) slot[nt + i] = slot[ndrop + i];
        }
        total = nt + (a.counts[sc] - ndrop);
    }
    for (int32_t i = 0; i < nt && i < a.capseg; ++i) slot[i] = scratch[i];
    a.counts[sc] = total;
}

// Re-run segment s of channel c from the true state T and the speculative state S0 side by side.
// Returns true if they merged; T becomes the true state at the segment end when they did not.
__device__ bool rerun_segment(const TrigSpecArgs& a, int c, int s, const int32_t (&tap)[kFirTaps],
                              const TrigCfg& k, TrigState& T, const TrigState& S0) {
    const int64_t seg0 = (int64_t)s * a.L;
    const int64_t seg1 = seg0 + a.L < a.J ? seg0 + a.L : a.J;
    uint64_t* scratch = a.scratch + (int64_t)c * a.capseg;
    TrigState tru = T, spc = S0;
    int32_t nt = 0, ndrop = 0;
    bool merged = false;
    Win win;
    load_window(win, a, c, seg0);
    const int16_t* rp = a.raw + seg0 * a.C + c;
    for (int64_t g = seg0; g < seg1 && !merged; g += kFirTaps) {
        const int64_t left = seg1 - g;
        // one latency per 26 samples: the group's loads are issued before the merge test can
        // stop the walk (a serial walk otherwise waits on every load)
        int32_t r[kFirTaps];
#pragma unroll
        for (int u = 0; u < kFirTaps; ++u) r[u] = u < left ? rp[(int64_t)u * a.C] : 0;
        rp += (int64_t)kFirTaps * a.C;
#pragma unroll
        for (int u = 0; u < kFirTaps; ++u) {
            if (u >= left || merged) continue;
            const int64_t j = g + u;
            win.w[u] = r[u];
            const int32_t f = mf_at(win, tap, u);
            uint64_t pkt;
            if (trig_step(tru, f, k, c, a.j0 + j, &pkt)) {
                if (nt < a.capseg) scratch[nt] = pkt;
                ++nt;
            }
            uint64_t dummy;
            if (trig_step(spc, f, k, c, a.j0 + j, &dummy)) ++ndrop;
            merged = state_eq(tru, spc, a.mode);
        }
    }
    if (!merged) T = tru;
    splice_segment(a, c, s, nt, ndrop, merged, scratch);
    return merged;
}

// SVF re-run of segment s of channel c on one wave (the filter pre-pass, a.filt): lanes 0 and 1
// step the true (from T) and the speculative (from S0) trajectory in lockstep (one instruction
// stream for both, the hot-loop form trig_update_svf) over the pre-filtered rows, 64 rows per
// block: each lane loads one row's f a block ahead and the walk broadcasts them with v_readlane.
// The merge is tested once per block (splice_segment). Lane 0 writes the true packets to out;
// nt / ndrop / merged are uniform, Tend (the true end state when not merged) is uniform.
// Round 5's single-lane walk (two generic trig_step per sample plus the 26-tap filter from raw
// rows) took 3.2 ms for one segment of 16384 rows at config 3; this one 0.71 ms.
__device__ bool svf_walk(const TrigSpecArgs& a, int c, int s, const TrigCfg& k, const TrigState& T,
                         const TrigState& S0, int lane, uint64_t* out, int32_t& nt, int32_t& ndrop, TrigState& Tend) {
    const int64_t seg0 = (int64_t)s * a.L;
    const int64_t seg1 = seg0 + a.L < a.J ? seg0 + a.L : a.J;
    const FastCfg q = fast_cfg(k);
    FastSvf st = to_fast_svf(lane == 0 ? T : S0);
    nt = 0;
    ndrop = 0;
    bool merged = false;
    const int16_t* fp = a.filt + c;
    // per block: each lane's emits as a bit mask (no per-row ballot and branch: the row loop is
    // the update chain alone), the compared baselines in LDS (lanes 1-63 run the same speculative
    // trajectory, so they store the same value), the packets assembled after the block
    __shared__ int32_t bsh[4][2][64];
    int32_t* bl = bsh[threadIdx.x >> 6][lane == 0 ? 0 : 1];
    int32_t fnext = seg0 + lane < seg1 ? (int32_t)fp[(seg0 + lane) * a.C] : 0;
    for (int64_t g = seg0; g < seg1 && !merged; g += 64) {
        const int32_t fl = fnext;
        // this block's rows arrived during the previous block: wait for them here, before the next
        // block's load is issued (a wait inside the row loop would also wait for that load)
        asm volatile("" ::"v"(fl));
        const int left = __builtin_amdgcn_readfirstlane((int)(seg1 - g < 64 ? seg1 - g : 64));
        fnext = g + 64 + lane < seg1 ? (int32_t)fp[(g + 64 + lane) * a.C] : 0;   // next block in flight
        const int32_t pf1 = __builtin_amdgcn_readlane(st.f1, 0), pf2 = __builtin_amdgcn_readlane(st.f2, 0);
        uint64_t em = 0;
        for (int i = 0; i < left; ++i) {
            const int32_t f = __builtin_amdgcn_readlane(fl, i);
            EvInfo ev;
            const bool e = trig_update_svf(st, f, q, a.kf, a.kq, ev);
            em |= (uint64_t)e << i;
            bl[i] = ev.base;
        }
        __builtin_amdgcn_wave_barrier();
        const uint64_t e0 = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int32_t)(em >> 32), 0) << 32) |
                            (uint32_t)__builtin_amdgcn_readlane((int32_t)em, 0);
        const uint64_t e1 = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int32_t)(em >> 32), 1) << 32) |
                            (uint32_t)__builtin_amdgcn_readlane((int32_t)em, 1);
        ndrop += __builtin_popcountll(e1);
        for (uint64_t m = e0; m; m &= m - 1) {   // lane 0's packets: row i, samples i - 2 .. i
            const int i = __builtin_ctzll(m);
            const int32_t f = __builtin_amdgcn_readlane(fl, i);
            const int32_t y2 = i >= 1 ? __builtin_amdgcn_readlane(fl, i - 1) : pf1;
            const int32_t y1 = i >= 2 ? __builtin_amdgcn_readlane(fl, i - 2) : (i == 1 ? pf1 : pf2);
            if (lane == 0 && nt < a.capseg) out[nt] = make_packet(c, EvInfo{y1, y2, bsh[threadIdx.x >> 6][0][i]}, f, a.j0 + g + i);
            ++nt;
        }
        __builtin_amdgcn_wave_barrier();
        auto same = [&](int32_t v) { return __builtin_amdgcn_readlane(v, 0) == __builtin_amdgcn_readlane(v, 1); };
        merged = same((int32_t)st.low) && same((int32_t)(st.low >> 32)) && same((int32_t)st.band) &&
                 same((int32_t)(st.band >> 32)) && same(st.x) && same(st.f1) && same(st.f2);
    }
    if (!merged) {   // lane 0's trajectory, broadcast
        FastSvf t;
        t.low = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int32_t)(st.low >> 32), 0) << 32) |
                          (uint32_t)__builtin_amdgcn_readlane((int32_t)st.low, 0));
        t.band = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int32_t)(st.band >> 32), 0) << 32) |
                           (uint32_t)__builtin_amdgcn_readlane((int32_t)st.band, 0));
        t.x = __builtin_amdgcn_readlane(st.x, 0);
        t.f1 = __builtin_amdgcn_readlane(st.f1, 0);
        t.f2 = __builtin_amdgcn_readlane(st.f2, 0);
        Tend = from_fast_svf(t);
    }
    return merged;
}

// The two-lane walk usable from any state: a start-of-stream state (hold-off, no baseline) takes
// the generic single-lane walk instead (rerun_segment). Called by every lane with T uniform; on
// return T is uniform (the true end state when the trajectories did not merge).
__device__ bool rerun_segment_svf(const TrigSpecArgs& a, int c, int s, const int32_t (&tap)[kFirTaps],
                                  const TrigCfg& k, TrigState& T, const TrigState& S0, int lane) {
    __shared__ TrigState t_sh;
    __shared__ int32_t m_sh;
    if (!T.binit || !S0.binit || in_holdoff(T) || in_holdoff(S0)) {   // start of stream: generic walk
        if (lane == 0) {
            TrigState t = T;
            m_sh = rerun_segment(a, c, s, tap, k, t, S0) ? 1 : 0;
            t_sh = t;
        }
        __syncthreads();
        const bool merged = m_sh != 0;
        T = t_sh;
        __syncthreads();
        return merged;
    }
    uint64_t* scratch = a.scratch + (int64_t)c * a.capseg;
    int32_t nt, ndrop;
    TrigState Tend = T;
    const bool merged = svf_walk(a, c, s, k, T, S0, lane, scratch, nt, ndrop, Tend);
    if (lane == 0) splice_segment(a, c, s, nt, ndrop, merged, scratch);
    if (!merged) T = Tend;
    __syncthreads();   // lane 0's slot and scratch writes before any later segment's re-run
    return merged;
}

// Phase A of the SVF fix-up (round 6): one wave per (channel c, segment s >= 1) of the sub-chunk.
// A segment whose speculated start state differs from its predecessor's speculative end state is
// re-run at once, assuming that end state is the true one (it is unless the predecessor itself
// fails and does not merge), into its own result and packet entries; k_trig_fix confirms the
// assumptions channel by channel and splices. The failed segments of all channels walk in parallel
// instead of one after another in their channel's wave.
__global__ __launch_bounds__(256) void k_trig_refix(TrigSpecArgs a) {
    const int C = a.C;
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (w >= (int64_t)C * (a.nseg - 1)) return;   // wave-uniform
    const int c = (int)(w % C), s = (int)(w / C) + 1;
    const int64_t sc = (int64_t)c * a.seg_stride + a.seg_off + s;
    RefixRes* res = a.refix + sc;
    const TrigState P = a.s_end[seg_state(a, c, s - 1)];
    const TrigState S0 = a.s_spec[seg_state(a, c, s)];
    int32_t status = RF_OK, nt = 0, ndrop = 0;
    TrigState Tend = P;
    if (!state_eq(P, S0, a.mode)) {
        if (!P.binit || !S0.binit || in_holdoff(P) || in_holdoff(S0)) {
            status = RF_SERIAL;   // start of stream: k_trig_fix walks it
        } else {
            const TrigCfg k{a.thr[c], a.rearm[c], a.mode, a.alpha, a.kf, a.kq, a.base_thr, a.dead};
            status = svf_walk(a, c, s, k, P, S0, lane, a.refix_pk + sc * a.capseg, nt, ndrop, Tend) ? RF_MERGED
                                                                                                  : RF_UNMERGED;
        }
    }
    if (lane == 0) {
        res->status = status;
        res->nt = nt;
        res->ndrop = ndrop;
        res->T = Tend;
    }
}

__global__ __launch_bounds__(64) void k_trig_fix(TrigSpecArgs a) {
    extern __shared__ uint64_t okbits[];  // bit s%64 of word s/64: segment s needs no re-run
    const int c = blockIdx.x;
    const int lane = threadIdx.x;
    const int nwords = (a.nseg + 63) / 64;
    // four words (256 boundaries) per batch, every state loaded whole and unconditionally (clamped
    // index; consecutive lanes read consecutive entries of the channel-major layout) so that the
    // batch's loads are in flight together, then compared without branches
    for (int wd0 = 0; wd0 < nwords; wd0 += 4) {
        bool ok[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int s = (wd0 + i) * 64 + lane;
            const bool valid = s >= 1 && s < a.nseg;
            const int64_t ie = seg_state(a, c, valid ? s - 1 : 0), ip = seg_state(a, c, valid ? s : 0);
            const TrigState e = a.s_end[ie];   // segment 0's entries when not valid (nseg >= 1)
            const TrigState p = a.s_spec[ip];
            ok[i] = !valid || state_eq_nb(e, p, a.mode);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint64_t b = __ballot(ok[i]);
            if (lane == 0 && wd0 + i < nwords) okbits[wd0 + i] = b;
        }
    }
    __syncthreads();
    // SVF with the filter pre-pass: the whole wave runs the control below (uniform) and the
    // re-runs use two lanes (rerun_segment_svf); otherwise lane 0 alone walks
    const bool wave_walk = a.mode == MKID_BASE_SVF && a.filt != nullptr;
    if (!wave_walk && lane != 0) return;
    int32_t tap[kFirTaps];
#pragma unroll
    for (int i = 0; i < kFirTaps; ++i) tap[i] = a.fir[c * kFirTaps + i];
    const TrigCfg k{a.thr[c], a.rearm[c], a.mode, a.alpha, a.kf, a.kq, a.base_thr, a.dead};
    int32_t reruns = 0;
    if (wave_walk && a.refix && a.refix_pk) {
        // phase B after k_trig_refix: walk the segments in order. While the true start of segment s
        // is s_end[s - 1] (truth), its phase-A result holds: OK keeps the speculative list, a re-run
        // is spliced, an unmerged one hands its true end state on. Otherwise (T) the segment is
        // checked against T and, if it differs, re-run here from T (phase A assumed the wrong start).
        bool truth = true;
        TrigState T{};
        for (int s = 1; s < a.nseg; ++s) {
            const int64_t sc = (int64_t)c * a.seg_stride + a.seg_off + s;
            const RefixRes* r = a.refix + sc;
            const int32_t st = r->status;
            const TrigState S0 = a.s_spec[seg_state(a, c, s)];
            if (truth) {
                if (st == RF_OK) continue;
                ++reruns;
                if (st == RF_MERGED || st == RF_UNMERGED) {
                    if (lane == 0) splice_segment(a, c, s, r->nt, r->ndrop, st == RF_MERGED, a.refix_pk + sc * a.capseg);
                    if (st == RF_UNMERGED) {
                        T = r->T;
                        truth = false;
                    }
                    continue;
                }
                T = a.s_end[seg_state(a, c, s - 1)];   // RF_SERIAL
                truth = rerun_segment_svf(a, c, s, tap, k, T, S0, lane);
            } else {
                if (state_eq(T, S0, a.mode)) {
                    truth = true;
                    continue;
                }
                ++reruns;
                truth = rerun_segment_svf(a, c, s, tap, k, T, S0, lane);
            }
        }
        if (lane != 0) return;
        a.st_out[c] = truth ? a.s_end[seg_state(a, c, a.nseg - 1)] : T;
        if (a.reruns) a.reruns[c] = reruns;
        return;
    }
    TrigState T{};
    bool override_ = false;  // T holds the true start state of segment s (from an unmerged re-run)
    int s = 1;
    while (s < a.nseg) {
        if (!override_) {
            // next segment whose precomputed check failed
            int wd = s >> 6;
            uint64_t fail = ~okbits[wd] & (~0ull << (s & 63));
            while (!fail && ++wd < nwords) fail = ~okbits[wd];
            if (!fail) break;
            s = wd * 64 + __builtin_ctzll(fail);
            if (s >= a.nseg) break;
            T = a.s_end[seg_state(a, c, s - 1)];
        } else if (state_eq(T, a.s_spec[seg_state(a, c, s)], a.mode)) {
            override_ = false;
            ++s;
            continue;
        }
        ++reruns;
        const TrigState S0 = a.s_spec[seg_state(a, c, s)];
        override_ = wave_walk ? !rerun_segment_svf(a, c, s, tap, k, T, S0, lane) : !rerun_segment(a, c, s, tap, k, T, S0);
        ++s;
    }
    if (lane != 0) return;
    a.st_out[c] = override_ ? T : a.s_end[seg_state(a, c, a.nseg - 1)];
    if (a.reruns) a.reruns[c] = reruns;
}

int64_t trigger_wave_slots(int device) {
    int ncu = 0, nb = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || ncu <= 0)
        ncu = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_trig_spec<MKID_BASE_EMA>, kSpecThreads, 0) != hipSuccess ||
        nb <= 0)
        nb = 1;
    return (int64_t)ncu * nb * (kSpecThreads / 64);
}

hipError_t launch_trigger(const TrigSpecArgs& a, hipStream_t s) {
    const int64_t threads = (int64_t)a.C * a.nseg;
    const dim3 grid((unsigned)((threads + kSpecThreads - 1) / kSpecThreads));
    if (a.mode == MKID_BASE_EMA)
        hipLaunchKernelGGL(k_trig_spec<MKID_BASE_EMA>, grid, dim3(kSpecThreads), 0, s, a);
    else if (a.mode == MKID_BASE_SVF && a.filt) {
        // filter pre-pass: row blocks of >= 520 rows (a multiple of 26), ~3 waves per SIMD
        const int64_t nt = std::max<int64_t>(1, (int64_t)3072 * 64 / a.C);
        int64_t rp = std::max<int64_t>(520, (a.J + nt - 1) / nt);
        rp = (rp + kFirTaps - 1) / kFirTaps * kFirTaps;
        const int64_t mthreads = (int64_t)a.C * ((a.J + rp - 1) / rp);
        hipLaunchKernelGGL(k_mf_rows, dim3((unsigned)((mthreads + kSpecThreads - 1) / kSpecThreads)),
                           dim3(kSpecThreads), 0, s, a, (int32_t)rp);
        hipError_t e0 = hipGetLastError();
        if (e0 != hipSuccess) return e0;
        hipLaunchKernelGGL((k_trig_spec<MKID_BASE_SVF, true>), grid, dim3(kSpecThreads), 0, s, a);
        if (a.refix && a.refix_pk && a.nseg > 1) {
            hipError_t e1 = hipGetLastError();
            if (e1 != hipSuccess) return e1;
            const int64_t waves = (int64_t)a.C * (a.nseg - 1);
            hipLaunchKernelGGL(k_trig_refix, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, s, a);
        }
    } else if (a.mode == MKID_BASE_SVF)
        hipLaunchKernelGGL(k_trig_spec<MKID_BASE_SVF>, grid, dim3(kSpecThreads), 0, s, a);
    else
        hipLaunchKernelGGL(k_trig_spec<MKID_BASE_NONE>, grid, dim3(kSpecThreads), 0, s, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const size_t lds = (size_t)((a.nseg + 63) / 64) * 8;
    hipLaunchKernelGGL(k_trig_fix, dim3(a.C), dim3(64), lds, s, a);
    return hipGetLastError();
}

}  // namespace mkid
