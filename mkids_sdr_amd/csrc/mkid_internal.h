// Internal declarations shared by the HIP translation units of libmkidgpu.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <string>
#include <vector>

#include "mkidgpu.h"

namespace mkid {

constexpr int kPfbTaps = 4;    // T: PFB taps per branch (build decision)
constexpr int kFirTaps = 26;   // ROACH_Pulses.py:61
constexpr int kLpfHist = kFirTaps - 2;  // z frames carried for the decimating IQ low-pass
constexpr int kRawHist = kFirTaps - 1;  // raw phase samples carried for the matched filter
// Start-of-stream trigger hold-off (phase samples): after a reset the trigger is DEAD with no
// baseline while the PFB / low-pass / matched-filter histories fill (build decision, DESIGN.md §2;
// oracle/trigger.c HOLDOFF)
constexpr int kHoldOff = 64;

// Per-channel trigger state. Byte layout identical to oracle/trigger.c trig_state.
struct TrigState {
    int32_t B, binit, st, cnt, f1, f2, pad0, pad1;
    int64_t low, band;
};
static_assert(sizeof(TrigState) == 48, "TrigState layout");

struct LpfTaps { float g[kFirTaps]; };

// IQ snapshot sample: the low-pass output in ADC-count units, rounded and saturated to int16
__device__ __forceinline__ int16_t iq16(float v) {
    const float r = rintf(v);
    return (int16_t)(r < -32768.f ? -32768.f : (r > 32767.f ? 32767.f : r));
}

struct ChanArgs {
    const uint32_t* x;      // chunk, int16 I/Q packed per 32-bit word
    const uint32_t* xhist;  // T*N - M previous samples
    const float* pfb;       // T*N prototype
    const int32_t* bins;    // C
    const float2* lo;       // [P][C], conj(LUT)/2^15
    float2* z;              // [K][C]
    int64_t K;              // frames in this chunk
    int64_t k0;             // global index of the chunk's first frame
    int32_t P;              // LO period (power of two)
    int32_t pad;
    int64_t frames_per_block;  // set by the launcher
    int64_t avail;          // samples readable before x (earlier sub-chunks of the same call);
                            // older samples come from xhist
};

// Centred low-pass (K5-K6 with the IQ-loop centre c subtracted BEFORE the accumulation, DESIGN.md
// §4): the kernels accumulate y' = sum_i g_i (z_i - c') with c' = c / G (G = sum_i g_i) and output
// phase = atan2(y' + r), r = G c' - c (host, float64). The partial sums then stay at the loop's
// radius instead of the tone's |y|, so the fp32 rounding of the accumulation no longer grows with
// |c| / radius. y = y' + (r + c) where the raw IQ is needed (IQ tap: `tap_off`; avgIQ: the host).
struct Centring {
    const float2* ncen;     // [C] -c' (the DDC's fused add)
    const float2* cor;      // [C] r
    float2 tap_off;         // r + c of the IQ-tap channel
};

struct LpfArgs {
    const float2* z;        // [K][C]
    const float2* zhist;    // [24][C]
    Centring cen;
    float* phase;           // [J][C] or nullptr
    int16_t* raw;           // [J][C]
    long long* ysum;        // [C][2] per-channel sum of y' (avgIQ), fixed point 2^-kYsumFrac, or nullptr
    int64_t J;
    int32_t C;
    LpfTaps taps;
    int16_t* iqtap;         // [J][2] int16 low-pass output of channel iq_ch (IQ snapshot) or nullptr
    int32_t iq_ch;
};

// avgIQ accumulator (firmware K9, avgIQ_bram): per-thread float partial sums are rounded to
// fixed point (2^-8) and added with integer atomics, so the sums do not depend on the order in
// which workgroups finish (float atomics would make the loop calibration run-to-run different)
constexpr int kYsumFrac = 8;
__device__ __forceinline__ void ysum_add(long long* ysum, int c, float sx, float sy) {
    atomicAdd(reinterpret_cast<unsigned long long*>(ysum) + 2 * c,
              (unsigned long long)llrintf(sx * (float)(1 << kYsumFrac)));
    atomicAdd(reinterpret_cast<unsigned long long*>(ysum) + 2 * c + 1,
              (unsigned long long)llrintf(sy * (float)(1 << kYsumFrac)));
}

struct FrontArgs {
    const uint32_t* x;      // chunk, int16 I/Q packed per 32-bit word
    const uint32_t* xhist;  // front_hist_samples(N) previous samples
    const uint2* pfbq;      // [N] int16 taps {h0|h1<<16, h2|h3<<16} of point p (scale 2^S in lo)
    const int32_t* bins;    // C
    const float2* lo;       // [P][C], conj(LUT)/2^15
    Centring cen;
    float* phase;           // [K/2][C] or nullptr
    int16_t* raw;           // [K/2][C]
    long long* ysum;        // [C][2] sums of y', fixed point 2^-kYsumFrac, or nullptr (accumulator off)
    int64_t K;              // frames in this chunk (even)
    int64_t k0;             // global index of the chunk's first frame
    int64_t frames_per_block;  // set by the launcher
    int64_t avail;          // samples readable before x (earlier sub-chunks of the same call)
    int32_t P;              // LO period (power of two)
    int32_t ncu;            // compute units of the device (grid sizing: per-CU multipliers)
    LpfTaps taps;
    int16_t* iqtap;         // [K/2][2] int16 low-pass output of channel iq_ch (IQ snapshot) or nullptr
    int32_t iq_ch;
    int32_t pad;
    const int16_t* slot_ch; // [C] k_front3 (N = 2048): channel of select slot st + 512 q (nullptr: identity)
};

// Result of one segment's parallel SVF re-run (k_trig_refix, round 6): status and, for a re-run,
// the true packets before the merge detection (in TrigSpecArgs::refix_pk at the segment's slot
// entry), the speculative packets the re-run dropped, and the true end state when it did not merge.
enum { RF_OK = 0, RF_MERGED = 1, RF_UNMERGED = 2, RF_SERIAL = 3 };
struct RefixRes {
    int32_t status, nt, ndrop, pad;
    TrigState T;
};
static_assert(sizeof(RefixRes) == 64, "RefixRes layout");

struct TrigSpecArgs {
    const int16_t* raw;     // [J][C] Fix16_13 phase
    const int16_t* rhist;   // [25][C] previous call's last raw samples
    const int16_t* fir;     // [C][26] matched-filter taps (int12)
    const int32_t* thr;     // [C]
    const int32_t* rearm;   // [C] re-arm levels (mkid_set_rearm; = thr without hysteresis)
    const TrigState* st_in; // [C] carried state (segment 0 starts from it)
    TrigState* st_out;      // [C] carried state after this call (may alias st_in)
    TrigState* s_spec;      // [C][nseg] speculative state at each segment start (k_trigger.hip seg_state)
    TrigState* s_end;       // [C][nseg] state at each segment end
    uint64_t* slots;        // [C][seg_stride][capseg] packets (entry c*seg_stride + seg_off + s)
    int32_t* counts;        // [C][seg_stride]
    uint64_t* scratch;      // [C][capseg] fix-up scratch
    int32_t* reruns;        // [C] segments re-run by the fix-up (diagnostic, nullable)
    int64_t J;
    int64_t j0;             // global index of the chunk's first phase sample
    int32_t C, nseg, L, W, capseg;
    int32_t mode, alpha, kf, kq, base_thr, dead;
    // the segments of one call's sub-chunks share one [C][seg_stride] slot table, so that a single
    // compaction at the end of the call orders packets channel-major over the whole call
    int32_t seg_stride, seg_off;
    // [J][C] matched-filter output (int16) of the SVF path's filter pre-pass (k_mf_rows), so
    // that the SVF walk, bound by one wave's instruction stream, skips the 26-tap filter
    int16_t* filt = nullptr;
    // SVF with the pre-pass: every failed segment is re-run in parallel (k_trig_refix) assuming its
    // predecessor's speculative end state, into [C][seg_stride] results and a [C][seg_stride][capseg]
    // packet table; k_trig_fix then confirms the assumptions channel by channel
    RefixRes* refix = nullptr;
    uint64_t* refix_pk = nullptr;
};

struct HeightArgs {
    const float* phase;      // [rows][C] rad, global phase rows j0 .. j0 + rows - 1
    const uint64_t* events;  // [n] wide packets
    const float* coeff;      // [C][ncoeff] per-channel optimal filter
    float* heights;          // [n] out (NaN: window outside the rows or unknown channel)
    int64_t rows, j0, n;    // n: packets (or the bound on *d_n)
    int32_t C, ncoeff, pre;
    const int64_t* d_n;     // nullable: device packet count (min(*d_n, n) packets are processed)
    // carried phase history: rows j0 - hrows .. j0 - 1 ([hrows][C]), read for windows that start
    // before the call's first row (hrows = 0: none)
    const float* hist;
    int64_t hrows;
    int32_t ncu;            // compute units of the device (grid cap)
    int32_t pad;
};

// launchers (return hipError_t of the launch)
hipError_t launch_pulse_heights(const HeightArgs& a, hipStream_t s);
hipError_t launch_channelize(int N, const ChanArgs& a, hipStream_t s);
hipError_t launch_lpf_phase(const LpfArgs& a, hipStream_t s);
hipError_t launch_front(int N, const FrontArgs& a, hipStream_t s);
hipError_t launch_trigger(const TrigSpecArgs& a, hipStream_t s);
// resident wave slots of the speculative trigger kernel on a device (occupancy x CUs)
int64_t trigger_wave_slots(int device);

hipError_t launch_hist_roll(void* dst, const void* old_hist, const void* fresh, int64_t hist_rows,
                            int64_t fresh_rows, int64_t row_bytes, hipStream_t s);
// one history-roll job (k_hist_roll's arguments), for the rolls carried by the compaction launch
struct RollJob {
    void* dst;
    const void* old_hist;
    const void* fresh;
    int64_t hist_rows, fresh_rows, row_bytes;
};
// K8 compaction; roll1 / roll2 (or null) run as extra blocks of its gather launch
hipError_t launch_compact(const uint64_t* slots, const int32_t* counts, int64_t n_ent,
                          int32_t capseg, uint64_t* out, int64_t cap, int64_t* d_counts,
                          int64_t* scan_ws, const RollJob* roll1, const RollJob* roll2, hipStream_t s);
hipError_t launch_stream_copy(void* dst, const void* src, int64_t bytes, hipStream_t s);
hipError_t launch_synth(int16_t* out, int64_t n, int64_t n0, const int16_t* base,
                        const mkid_synth_tone* tones, const mkid_pulse* pulses, int64_t npulses,
                        float tr, float tf, int32_t window, float sigma, uint32_t seed,
                        hipStream_t s);

hipError_t launch_replay(const int16_t* raw, int64_t n, int64_t ld, int32_t nch, int32_t mode, int32_t length,
                         int64_t start, int64_t need, int64_t skip, int32_t wrap, double thr, uint32_t* flags,
                         double* means, int32_t* hits, int32_t cap, int32_t* counts, hipStream_t s);

hipError_t launch_make_template(float* I, float* Q, int64_t P, double* rows, double* nrows, int32_t* accept,
                                double* peaks, int32_t* appended, double* scratch, double* tP, double* tPf,
                                double* noise, double* stats, float* refmed, hipStream_t s);
hipError_t launch_optimal_filter(const double* tpl, const double* noise, int pre, int ncoeff, double* coeff,
                                 double* work, hipStream_t s);

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (kernel, device), thread-safe: the
// attribute is per device, and several contexts (devices, host threads) may launch concurrently.
// `mask` is one static per kernel instantiation; the call is idempotent, so a race only repeats it.
inline hipError_t ensure_lds_attr(std::atomic<uint64_t>& mask, const void* fn, int bytes) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const uint64_t bit = 1ull << (dev & 63);
    if (mask.load(std::memory_order_acquire) & bit) return hipSuccess;
    e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e == hipSuccess) mask.fetch_or(bit, std::memory_order_acq_rel);
    return e;
}

bool channelize_supported(int N);
// fused PFB..phase front ends: k_front (N = 128 / 256), k_front3 (512 / 1024 / 2048, wave-
// specialised), k_front5 (4096, wave-specialised); fused_supported / launch_fused dispatch by N
bool fused_supported(int N);
hipError_t launch_fused(int N, const FrontArgs& a, hipStream_t s);
hipError_t launch_front(int N, const FrontArgs& a, hipStream_t s);   // N = 128 / 256 (k_front.hip)
hipError_t launch_front3(int N, const FrontArgs& a, hipStream_t s);  // N = 512 / 1024 / 2048 (k_front3.hip)
hipError_t launch_front5(const FrontArgs& a, hipStream_t s);         // N = 4096 (k_front5.hip)
int64_t front_hist_samples(int N);  // ADC history the fused kernel reads before a chunk

}  // namespace mkid
