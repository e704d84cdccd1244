// Host-side planning (mkid_plan.h): plain C++, no HIP, built into libmkidgpu.so and, with
// -fsanitize=address,undefined, into the CPU fuzz driver tools/plan_fuzz.cpp.
#include <array>
#include "mkid_plan.h"

#include <algorithm>
#include <climits>
#include <cmath>

namespace mkid {
namespace plan {

int64_t seg_capacity(int64_t L, int dead) { return L / (dead + 3) + 2; }

int64_t seg_length(int64_t J, int C, int64_t wave_slots) {
    const int64_t nt = std::max<int64_t>(1, wave_slots * 64 / C);
    return std::max<int64_t>(kSegL, (J + nt - 1) / nt);
}

const char* size_workspace(const mkid_cfg& cfg, bool fused, int64_t trig_slots, int64_t svf_lanes,
                           int64_t svf_w, Workspace& ws) {
    const int C = cfg.n_channels, N = cfg.fft_len;
    if (C <= 0 || N != 2 * C || cfg.max_chunk < N || cfg.max_chunk % N != 0 || cfg.dead_time < 0)
        return "unsupported geometry";
    if (trig_slots < 1 || svf_lanes < 1 || svf_w < kFirTaps || svf_w % kFirTaps != 0) return "bad tuning values";
    ws = Workspace{};
    // split front end: a large call is cut into 4 sub-chunks so the channeliser (stream A) of
    // sub-chunk i+1 overlaps the low-pass/trigger (stream B) of sub-chunk i
    int64_t G = cfg.max_chunk;
    if (!fused && G >= (int64_t)512 * N) {
        G = cfg.max_chunk / 4;
        G -= G % N;
    }
    ws.max_chunk = cfg.max_chunk;
    ws.G = G;
    ws.Kmax = G / (N / 2);
    ws.Jmax = G / N;
    ws.nsub_max = (cfg.max_chunk + G - 1) / G;
    ws.trig_slots = trig_slots;
    ws.svf_lanes = svf_lanes;
    ws.svf_w = svf_w;
    // packet capacities are hard bounds (seg_capacity): no per-channel/segment overflow can occur
    const int64_t cap_bound = seg_capacity(ws.Jmax, cfg.dead_time);   // whole sub-chunk, one segment
    ws.capc = std::min<int64_t>(cfg.max_events_per_ch > 0 ? cfg.max_events_per_ch : cap_bound, INT_MAX / 2);
    // plan_sub rounds segment lengths UP to the 26-sample ring: every segment of a sub-chunk of
    // J <= Jmax rows is at most round26(Jmax) long (EMA: round26(max(kSegL, ceil(J / nt))), and a
    // multi-segment plan needs J > kSegL; SVF: round26(ceil(J / nseg)) or J), and the EMA segments of
    // a full sub-chunk at most Lmax = round26(seg_length(Jmax)) (found by tools/plan_fuzz.cpp: sizing
    // from the unrounded lengths left some legal calls one packet short of the scratch)
    auto round26 = [](int64_t L) { return (L + kFirTaps - 1) / kFirTaps * kFirTaps; };
    const int64_t Lmax = round26(seg_length(ws.Jmax, C, trig_slots));
    // for J <= Jmax: L(J) <= Lmax and ceil(J / L(J)) <= max(slots * 64 / C, ceil(Jmax / kSegL))
    ws.nseg_max = std::max<int64_t>(std::max<int64_t>(1, trig_slots * 64 / C), (ws.Jmax + kSegL - 1) / kSegL);
    const int64_t capseg = seg_capacity(Lmax, cfg.dead_time);
    const int64_t capseg_any = seg_capacity(round26(ws.Jmax), cfg.dead_time);   // any one segment
    // one [C][sum of the sub-chunks' segments][capseg] table per call (single compaction)
    ws.slot_cap = (int64_t)C * ws.nsub_max * std::max<int64_t>(std::max<int64_t>(ws.nseg_max * capseg, ws.capc), capseg_any);
    // the fix-up re-runs one segment per channel into [C][capseg]: any plan's capseg, including an
    // SVF segment as long as the whole sub-chunk (plan_sub), whatever max_events_per_ch says
    ws.scratch_cap = std::max<int64_t>(std::max<int64_t>(capseg, ws.capc), capseg_any);
    return nullptr;
}

SubPlan plan_sub(const Workspace& ws, int C, int mode, int dead, int64_t J) {
    SubPlan p;
    p.J = J;
    if (mode == MKID_BASE_SVF) {
        // svf_lanes segments over all channels (the per-lane walk is latency bound), each
        // >= kSvfLmin rows; short sub-chunks run as one exact segment
        const int64_t want = std::max<int64_t>(1, ws.svf_lanes / C);
        const int64_t nseg = std::min<int64_t>(std::min<int64_t>(want, J / kSvfLmin), ws.nseg_max);
        p.W = 0;
        p.L = (int32_t)J;
        p.nseg = 1;
        if (nseg > 1 && J > 2 * kSvfLmin) {
            int64_t L = (J + nseg - 1) / nseg;
            L = (L + kFirTaps - 1) / kFirTaps * kFirTaps;
            p.L = (int32_t)L;
            p.W = (int32_t)ws.svf_w;
            p.nseg = (int32_t)((J + L - 1) / L);
        }
        p.capseg = (int32_t)seg_capacity(p.L, dead);
        return p;
    }
    const bool serial = J <= kSegL;
    // segment starts at multiples of 26 (the trigger's window ring is group-aligned)
    const int64_t Ls = serial ? J : (seg_length(J, C, ws.trig_slots) + kFirTaps - 1) / kFirTaps * kFirTaps;
    p.L = (int32_t)Ls;
    p.W = serial ? 0 : (int32_t)kSegW;
    p.nseg = (int32_t)((J + Ls - 1) / Ls);
    p.capseg = (int32_t)seg_capacity(Ls, dead);
    return p;
}

const char* plan_call(const Workspace& ws, int C, int N, int mode, int dead, int64_t n,
                      std::vector<SubPlan>& subs, int32_t& stride, int32_t& capseg) {
    subs.clear();
    stride = 0;
    capseg = 1;
    // the per-call buffers (raw rows, IQ tap, slot table) hold max_chunk samples
    if (n <= 0 || n % N != 0 || n > ws.max_chunk) return "call size outside the workspace";
    for (int64_t off = 0; off < n; off += ws.G) {
        subs.push_back(plan_sub(ws, C, mode, dead, std::min<int64_t>(ws.G, n - off) / N));
        stride += subs.back().nseg;
        capseg = std::max(capseg, subs.back().capseg);
        if (subs.back().nseg > ws.nseg_max) return "trigger plan exceeds the segment tables";
    }
    if ((int64_t)C * stride * capseg > ws.slot_cap) return "trigger plan exceeds the packet slot table";
    if (capseg > ws.scratch_cap) return "trigger plan exceeds the fix-up scratch";
    return nullptr;
}

// Select-slot order (mkid_slot_order). A select thread reads, per channel and frame, the Y entry
// `key` of its bin in each region; a ds_read_b64 costs one LDS cycle per distinct address on the
// busiest bank pair of each 32-lane half (MI355X_MICROARCH.md §LDS), and entry e sits on pair
// e mod 32 (regions and frames are 0 mod 32 entries apart). Each select wave's channels are
// spread over its read groups (one per half-wave and read instruction) so that a group's 32
// channels fall on distinct pairs where the bins allow, each wave keeping its own channels (its
// stores and LO loads stay within the same lines). Greedy per wave: channels by pair-class size,
// each into the group whose cost rises least, then whose new cost is lowest, then the emptiest
// (tools/lds_assign.py holds the same algorithm and its model).
//   k_front3, C = 1024 (N = 2048): key yswz(bin & 511); wave w owns channels 128 w .. 128 w + 127,
//     slot st + 512 q (st = 64 w + 32 h + l) is lane 32 h + l of wave w in read instruction q:
//     random bins ~3.4 cycles per group in channel order, ~1.9 ordered (PMC 287 M -> 156 M).
//   k_front5 layout, C = 2048 (N = 4096): key yswz(bin & 511) + 4 REG s (the pre-combined region
//     P^s, s = bit 9 of the bin: same pair, another address); select wave sw < 8 owns channels
//     64 sw + l + 512 q (q < 3, 6 groups), wave 8 + v owns 1536 + 64 v + l + 256 q (q < 2, 4 groups).
//     Computed for the model and tests only: applied in k_front5 (round 6) it cut the PMC LDS
//     conflict cycles 390.5 M -> 152.9 M per launch but took 2.5 % (plain stores) to 6 %
//     (non-temporal) more time, the scattered stores and the channel decoding costing more than
//     the conflicts, which sit off the transform waves' critical chain.
namespace {
void assign_groups(const std::vector<int>& yo, int ng, std::vector<std::vector<int>>& member) {
    constexpr int GS = 32;
    const int B = (int)yo.size();
    int cnt[32] = {0};
    for (int i = 0; i < B; ++i) ++cnt[yo[i] & 31];
    std::vector<int> order(B);
    for (int i = 0; i < B; ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
        const int ka = yo[a] & 31, kb = yo[b] & 31;
        if (cnt[ka] != cnt[kb]) return cnt[ka] > cnt[kb];
        if (ka != kb) return ka < kb;
        return yo[a] < yo[b];
    });
    std::vector<int> size(ng, 0), gmax(ng, 0);
    std::vector<std::array<int, 32>> mult(ng);
    for (auto& m : mult) m.fill(0);
    std::vector<std::vector<int>> seen(ng);
    member.assign(ng, {});
    for (int i : order) {
        const int k = yo[i] & 31;
        int bg = -1, bk0 = 0, bk1 = 0, bk2 = 0;
        bool bsame = false;
        for (int g = 0; g < ng; ++g) {
            if (size[g] >= GS) continue;
            const bool same = std::find(seen[g].begin(), seen[g].end(), yo[i]) != seen[g].end();
            const int m = mult[g][k] + (same ? 0 : 1);
            const int nm = std::max(gmax[g], m);
            const int k0 = nm - gmax[g], k1 = nm, k2 = size[g];
            if (bg < 0 || k0 < bk0 || (k0 == bk0 && (k1 < bk1 || (k1 == bk1 && k2 < bk2)))) {
                bg = g; bk0 = k0; bk1 = k1; bk2 = k2; bsame = same;
            }
        }
        member[bg].push_back(i);
        ++size[bg];
        if (!bsame) {
            seen[bg].push_back(yo[i]);
            ++mult[bg][k];
        }
        gmax[bg] = std::max(gmax[bg], mult[bg][k]);
    }
}

int yswz_entry(int b) {
    const int k = b & 511;
    return k ^ ((k >> 2) & 14);
}
}  // namespace

void slot_order(const std::vector<int32_t>& bins, int C, std::vector<int16_t>& out) {
    out.resize(C);
    for (int i = 0; i < C; ++i) out[i] = (int16_t)i;
    if ((C != 1024 && C != 2048) || (int)bins.size() < C) return;
    // per wave: the slots of its read groups (group j = read instruction j >> 1, half j & 1)
    struct Wave { int base, stride, nq; };
    std::vector<Wave> waves;
    if (C == 1024) {
        for (int w = 0; w < 8; ++w) waves.push_back({64 * w, 512, 2});
    } else {
        for (int w = 0; w < 8; ++w) waves.push_back({64 * w, 512, 3});
        for (int v = 0; v < 4; ++v) waves.push_back({1536 + 64 * v, 256, 2});
    }
    constexpr int kRegion4 = 4 * 576;   // k_front5: P^1 regions start 4 REG entries after P^0
    for (const Wave& wv : waves) {
        const int ng = 2 * wv.nq;
        // the wave's channels: k_front3 owns 128 consecutive channels (its slot order predates the
        // k_front5 one and is kept bit-identical); k_front5 the natural channels of its slots
        std::vector<int> chans;
        if (C == 1024) {
            const int w = wv.base / 64;
            for (int i = 0; i < 128; ++i) chans.push_back(128 * w + i);
        } else {
            for (int q = 0; q < wv.nq; ++q)
                for (int l = 0; l < 64; ++l) chans.push_back(wv.base + l + wv.stride * q);
        }
        std::vector<int> yo(chans.size());
        for (size_t i = 0; i < chans.size(); ++i) {
            const int b = bins[chans[i]];
            yo[i] = yswz_entry(b) + (C == 2048 ? kRegion4 * ((b >> 9) & 1) : 0);
        }
        std::vector<std::vector<int>> member;
        assign_groups(yo, ng, member);
        for (int g = 0; g < ng; ++g)
            for (int l = 0; l < 32; ++l)
                out[wv.base + 32 * (g & 1) + l + wv.stride * (g >> 1)] = (int16_t)chans[member[g][l]];
    }
}

// K1 taps as the device applies them (include/mkidgpu.h, mkid_set_pfb): h_q = rint(h 2^S) int16
// with the largest S such that every point's four |h_q| sum to <= 65535 and every |h_q| <= 32767
// (so the fused kernels' int16 dot products never overflow int32 on int16 samples).
int quantize_pfb(const float* h, int T, int N, std::vector<int16_t>& hq) {
    double ms = 0.0, ma = 0.0;
    for (int p = 0; p < N; ++p) {
        double sp = 0.0;
        for (int t = 0; t < T; ++t) {
            const double a = std::fabs((double)h[t * N + p]);
            sp += a;
            ma = std::max(ma, a);
        }
        ms = std::max(ms, sp);
    }
    int S = 0;
    if (ms > 0.0) {
        S = -64;
        while (S < 64 && std::ldexp(ms, S + 1) <= 65535.0 && std::ldexp(ma, S + 1) <= 32767.0) ++S;
    }
    hq.resize((size_t)T * N);
    // rounding can push a point's sum of |h_q| past 65535 (and a dot product of full-scale
    // samples past INT32_MAX): step S down until the ROUNDED taps obey both bounds
    for (;; --S) {
        bool ok = true;
        for (size_t i = 0; i < hq.size(); ++i) {
            const double r = std::rint(std::ldexp((double)h[i], S));
            if (std::fabs(r) > 32767.0) ok = false;
            hq[i] = ok ? (int16_t)r : 0;
        }
        for (int p = 0; p < N && ok; ++p) {
            int64_t sp = 0;
            for (int t = 0; t < T; ++t) sp += std::abs((int64_t)hq[(size_t)t * N + p]);
            if (sp > 65535) ok = false;
        }
        if (ok || S <= -64) break;
    }
    return S;
}

void merge_channel_major(uint64_t* ev, int64_t n) {
    if (n > 1)
        std::stable_sort(ev, ev + n, [](uint64_t a, uint64_t b) {
            return (a >> MKID_PKT_CH_SHIFT) < (b >> MKID_PKT_CH_SHIFT);
        });
}

int pack_reference(const uint64_t* wide, int64_t n, uint64_t* out) {
    for (int64_t i = 0; i < n; ++i) {
        const uint64_t w = wide[i];
        const uint64_t ch = (w >> MKID_PKT_CH_SHIFT) & 0xFFF;
        if (ch >= 255) return -1;  // 8-bit channel field, 255 = end-of-second marker
        const uint64_t pk = (w >> MKID_PKT_PEAK_SHIFT) & 0xFFF, bs = (w >> MKID_PKT_BASE_SHIFT) & 0xFFF;
        const uint64_t p1 = (uint64_t)std::min<int64_t>(4095, std::max<int64_t>(0, (int64_t)pk - (int64_t)bs + 2048));
        const uint64_t ts = w & 0xFFFFF;
        out[i] = (ch << 56) | (pk << 44) | (p1 << 32) | (bs << 20) | ts;
    }
    return 0;
}

int32_t rearm_level(int32_t thr, int32_t q8) {
    const int64_t p = (int64_t)thr * q8;
    const int64_t fl = p >= 0 ? p / 256 : -((-p + 255) / 256);   // floor(p / 256), no shift of a negative
    return (int32_t)((int64_t)thr - fl);
}

}  // namespace plan
}  // namespace mkid
