// Host-side planning of libmkidgpu.so, free of HIP so that it builds and runs on the CPU under
// AddressSanitizer / UndefinedBehaviorSanitizer (make -C mkids_sdr_amd/csrc asan; tools/plan_fuzz.cpp):
// workspace sizing at context creation, the per-call trigger segmentation and its slot-table
// geometry, the k_front3 select-slot order, the K1 tap quantisation, the merge of per-chunk packet
// lists and the reference packet re-encode. mkid_api.hip is the only product caller.
#pragma once
#include <stdint.h>

#include <vector>

#include "mkidgpu.h"

namespace mkid {
namespace plan {

constexpr int kFirTaps = 26;   // ROACH_Pulses.py:61
constexpr int kPfbTaps = 4;

// Speculative trigger segmentation (k_trigger.hip): segments of at least kSegL phase samples,
// each speculating from kSegW samples of warm-up (a multiple of the 26-sample matched-filter ring).
// The EMA baseline (alpha 41/512) forgets its start in ~10^2 samples on noisy phase. The warm-up is
// pure overhead when the speculation holds and the fix-up re-runs a segment when it does not
// (exact either way): on the bench stream 520 -> 260 samples is -6 % trigger time with no re-run,
// 130 re-runs 427 segments per step and gains nothing (profiles/r04/r04_j_kbench_trig_warmup.json).
// The floor kSegL only binds when the channels are few (256 at config 2: 2^28 samples give 2048
// rows per channel-segment at one wave per SIMD); 2048 -> 1024 is -41 % k_trig_spec there, 512
// no better, and config 3 / 5 segments are longer anyway (profiles/r04/r04_o_kbench_c2.json).
constexpr int64_t kSegL = 1024;
constexpr int64_t kSegW = 260;
// SVF baseline (Chamberlin 2-pole, Kf 82 / Kq 93623 Fix18_16): two integer trajectories started
// from different states coincide only after ~10^4 samples (median 1.5e4, 99th percentile 2.9e4, max
// 3.9e4 over 1024 simulated noisy channels; on the bench stream a 49k-sample warm-up misses 0.3 %
// of segments, 98k about 1 in 30000). Since round 6 the misses are re-run in
// parallel (k_trig_refix), so the warm-up is the half length: 49 140 samples with segments at one
// per SIMD lane (mkid_api.hip) measured 84-85 GS/s at config 3 against 65 for 98 280 at one per two
// lanes (profiles/r06/r06{f,g}_svf_*). Lengths are multiples of 26 so that every warm-up start keeps
// the filter ring aligned; segments are at least kSvfLmin long.
constexpr int64_t kSvfW = 26 * 1890;
constexpr int64_t kSvfLmin = 26 * 158;
static_assert(kSegW % kFirTaps == 0 && kSegL >= kSegW + kFirTaps - 1, "segment geometry");
static_assert(kSvfW % kFirTaps == 0, "SVF warm-up geometry");

// Packets a channel can produce in L phase rows: an event needs >= dead + 3 samples (trigger, peak,
// dead time, re-arm), plus the partial cycles at both ends.
int64_t seg_capacity(int64_t L, int dead);
// segment length for J rows: >= kSegL, and (C/64) * ceil(J/L) waves <= the resident wave slots
int64_t seg_length(int64_t J, int C, int64_t wave_slots);

// What a context was sized for (mkid_create): every later call is planned within it.
struct Workspace {
    int64_t max_chunk = 0;    // samples per call (cfg.max_chunk)
    int64_t G = 0;            // samples per sub-chunk (max_chunk, or max_chunk/4 on the split path)
    int64_t Kmax = 0, Jmax = 0, nsub_max = 0;
    int64_t capc = 0;         // per-channel packet capacity of a whole sub-chunk
    int64_t trig_slots = 0, svf_lanes = 0, svf_w = kSvfW;
    int64_t nseg_max = 0;     // segments per sub-chunk
    int64_t slot_cap = 0;     // packet slots of the [C][stride][capseg] table
    int64_t scratch_cap = 0;  // per-channel fix-up scratch
};
// cfg already validated (N = 2C, max_chunk a multiple of N, dead_time >= 0); ncu = compute units
const char* size_workspace(const mkid_cfg& cfg, bool fused, int64_t trig_slots, int64_t svf_lanes,
                           int64_t svf_w, Workspace& ws);

// Trigger geometry of one sub-chunk of J phase rows: segment length L, warm-up W, nseg segments and
// the per-segment packet capacity.
struct SubPlan {
    int64_t J;
    int32_t L, W, nseg, capseg;
};
SubPlan plan_sub(const Workspace& ws, int C, int mode, int dead, int64_t J);
// The sub-chunk plans of a call of n samples (n a positive multiple of N, n <= max_chunk) and the
// call's slot-table geometry: stride = total segments per channel, capseg = the largest per-segment
// capacity. Returns nullptr, or the error text when the plan exceeds the workspace.
const char* plan_call(const Workspace& ws, int C, int N, int mode, int dead, int64_t n,
                      std::vector<SubPlan>& subs, int32_t& stride, int32_t& capseg);

// k_front3 select-slot order (mkid_api.hip / include/mkidgpu.h mkid_slot_order): out[slot] = channel
void slot_order(const std::vector<int32_t>& bins, int C, std::vector<int16_t>& out);

// K1 taps as the device applies them: h_q = rint(h 2^S) int16, returns S
int quantize_pfb(const float* h, int T, int N, std::vector<int16_t>& hq);

// K7 re-arm level of a channel (mkid_set_rearm; oracle/trigger.py rearm_levels): the level moves
// from the threshold toward 0 (the baseline) by q8 / 256: thr - floor(thr q8 / 256), q8 in 0..256
int32_t rearm_level(int32_t thr, int32_t q8);

// per-chunk channel-major packet lists concatenated -> one channel-major list (stable in time)
void merge_channel_major(uint64_t* ev, int64_t n);

// wide device packet -> reference 64-bit packet; -1 if a channel does not fit the 8-bit field
int pack_reference(const uint64_t* wide, int64_t n, uint64_t* out);

}  // namespace plan
}  // namespace mkid
