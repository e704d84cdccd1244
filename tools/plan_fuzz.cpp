// CPU fuzz driver for the host planning code (mkids_sdr_amd/csrc/mkid_plan.cpp) and the oracle
// trigger (oracle/trigger.c), built with -fsanitize=address,undefined by
// `make -C mkids_sdr_amd/csrc asan` and run by tests/test_asan.py. Every check is an invariant the
// device code relies on (include/mkidgpu.h); the slot-table writes are replayed into
// buffers of exactly the planned size, so an undersized plan is an ASan heap overflow, not a
// silent miscount (the ADVICE r02 scratch-sizing bug is that class).
//   plan_fuzz [iterations] [seed]
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <random>
#include <vector>

#include "mkid_plan.h"

extern "C" {
typedef struct {
    int32_t B, binit, st, cnt, f1, f2, pad0, pad1;
    int64_t low, band;
} trig_state;
void oracle_trig_reset_state(trig_state* st, int32_t C);
int64_t oracle_trigger(const int16_t* raw, int64_t J, int32_t C, const int16_t* taps, const int32_t* thr,
                       const int32_t* rearm, int32_t mode,
                       int32_t alpha, int32_t kf, int32_t kq, int32_t base_thr, int32_t dead, int16_t* hist,
                       trig_state* st, int64_t j0, uint64_t* ev, int64_t cap, int64_t* counts);
}

using namespace mkid::plan;

static int failures = 0;
#define CHECK(cond, ...)                                        \
    do {                                                        \
        if (!(cond)) {                                          \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);                       \
            fprintf(stderr, "\n");                              \
            if (++failures > 20) exit(1);                       \
        }                                                       \
    } while (0)

static std::mt19937_64 rng;
static int64_t rint_(int64_t lo, int64_t hi) { return std::uniform_int_distribution<int64_t>(lo, hi)(rng); }

// workspace sizing + call plans for random geometries and ragged calls; the kernels' slot-table
// writes ([C][stride][capseg], per (channel, segment) at most seg_capacity(L) packets; fix-up scratch
// [C][capseg]) are replayed into exactly-sized buffers
static void fuzz_plans(int iters) {
    const int Cs[] = {64, 128, 256, 512, 1024, 2048};
    const int deads[] = {0, 1, 5, 32, 200};
    for (int it = 0; it < iters; ++it) {
        mkid_cfg cfg{};
        cfg.n_channels = Cs[rint_(0, 5)];
        cfg.fft_len = 2 * cfg.n_channels;
        const int C = cfg.n_channels, N = cfg.fft_len;
        cfg.pfb_taps = 4;
        cfg.fir_taps = 26;
        cfg.dds_entries = 65536 / C;
        cfg.dead_time = deads[rint_(0, 4)];
        const int me = (int)rint_(0, 3);
        cfg.max_events_per_ch = me == 0 ? 0 : (me == 1 ? 1 : (me == 2 ? 3 : (int)rint_(1, 5000)));
        // max_chunk: small (a few rows) to large (2^27 samples), sized so the replay stays small
        const int64_t rows_max = rint_(0, 3) == 0 ? rint_(1, 64) : rint_(1, std::max<int64_t>(1, (1 << 26) / N));
        cfg.max_chunk = rows_max * N;
        const bool fused = rint_(0, 1) == 1;
        const int64_t trig_slots = rint_(0, 2) == 0 ? rint_(1, 64) : rint_(1, 40000);
        const int64_t svf_lanes = rint_(0, 2) == 0 ? rint_(1, 100) : (rint_(0, 1) ? 256 * 256 : 256 * 128);
        const int64_t svf_w = 26 * rint_(1, 4000);
        Workspace ws;
        const char* e = size_workspace(cfg, fused, trig_slots, svf_lanes, svf_w, ws);
        CHECK(e == nullptr, "size_workspace failed: %s", e);
        if (e) continue;
        CHECK(ws.G > 0 && ws.G % N == 0 && ws.G * ws.nsub_max >= cfg.max_chunk, "sub-chunk geometry");
        CHECK(ws.nseg_max >= 1 && ws.slot_cap > 0 && ws.scratch_cap > 0, "table sizes");
        for (int call = 0; call < 6; ++call) {
            const int mode = (int)rint_(0, 2);
            // ragged calls: one row, all rows, a random count, one past the end
            int64_t rows;
            switch (call) {
                case 0: rows = 1; break;
                case 1: rows = rows_max; break;
                case 5: rows = rows_max + rint_(1, 3); break;
                default: rows = rint_(1, rows_max);
            }
            const int64_t n = rows * N;
            std::vector<SubPlan> subs;
            int32_t stride = 0, capseg = 0;
            const char* pe = plan_call(ws, C, N, mode, cfg.dead_time, n, subs, stride, capseg);
            if (n > cfg.max_chunk) {
                CHECK(pe != nullptr, "a call longer than max_chunk was planned");
                continue;
            }
            CHECK(pe == nullptr, "plan_call failed: %s (C %d rows %lld mode %d)", pe, C, (long long)rows, mode);
            if (pe) continue;
            int64_t Jsum = 0, segs = 0;
            for (const SubPlan& sp : subs) {
                Jsum += sp.J;
                segs += sp.nseg;
                CHECK(sp.J >= 1 && sp.J <= ws.Jmax, "sub-chunk rows %lld", (long long)sp.J);
                CHECK(sp.nseg >= 1 && sp.nseg <= ws.nseg_max, "nseg %d of %lld", sp.nseg, (long long)ws.nseg_max);
                CHECK(sp.L >= 1 && (int64_t)(sp.nseg - 1) * sp.L < sp.J && (int64_t)sp.nseg * sp.L >= sp.J,
                      "segments do not tile J: J %lld L %d nseg %d", (long long)sp.J, sp.L, sp.nseg);
                CHECK(sp.W >= 0 && sp.W % 26 == 0, "warm-up %d", sp.W);
                CHECK(sp.nseg == 1 || sp.L % 26 == 0, "segment starts off the 26-sample ring");
                CHECK(sp.capseg >= seg_capacity(sp.L, cfg.dead_time) && sp.capseg <= capseg, "capseg");
            }
            CHECK(Jsum == rows, "sub-chunks cover %lld of %lld rows", (long long)Jsum, (long long)rows);
            CHECK(segs == stride, "stride");
            CHECK((int64_t)C * stride * capseg <= ws.slot_cap, "slot table");
            CHECK(capseg <= ws.scratch_cap, "scratch");
            // replay the writes into exactly-sized tables (ASan catches any overrun)
            if (ws.slot_cap <= (int64_t)1 << 22 && (int64_t)C * ws.scratch_cap <= (int64_t)1 << 22) {
                std::vector<uint8_t> slots((size_t)ws.slot_cap), scratch((size_t)(C * ws.scratch_cap));
                const int64_t ch[] = {0, C - 1, rint_(0, C - 1)};
                int32_t seg_off = 0;
                for (const SubPlan& sp : subs) {
                    for (int64_t c : ch)
                        for (int32_t s = 0; s < sp.nseg; s += std::max<int32_t>(1, sp.nseg - 1)) {
                            const int64_t base = (c * stride + seg_off + s) * (int64_t)capseg;
                            for (int32_t k = 0; k < sp.capseg; k += std::max<int32_t>(1, sp.capseg - 1))
                                slots[(size_t)(base + k)] = 1;
                            for (int32_t k = 0; k < sp.capseg; k += std::max<int32_t>(1, sp.capseg - 1))
                                scratch[(size_t)(c * capseg + k)] = 1;
                        }
                    seg_off += sp.nseg;
                }
            }
        }
    }
}

// Sizing-only pass at the bench's scale: max_chunk up to 2^31 samples and the trigger
// slot / SVF lane counts of an MI355X (256 CUs; k_trig_spec at 4 blocks of 4 waves per CU; one SVF
// segment per two SIMD lanes), so SVF segments longer than the EMA segment the slot table was sized
// from are planned too. Every legal call (n <= max_chunk, n a multiple of N) must be accepted; no
// buffers are replayed (they would be GiB).
static void fuzz_sizing(int iters) {
    const int Cs[] = {256, 1024, 2048};
    const int deads[] = {0, 32, 200};
    const int64_t trig_slots = 256 * 4 * 4, svf_lanes = 256 * 256;   // an MI355X (mkid_api.hip)
    for (int it = 0; it < iters; ++it) {
        mkid_cfg cfg{};
        cfg.n_channels = Cs[rint_(0, 2)];
        cfg.fft_len = 2 * cfg.n_channels;
        const int C = cfg.n_channels, N = cfg.fft_len;
        cfg.pfb_taps = 4;
        cfg.fir_taps = 26;
        cfg.dds_entries = 65536 / C;
        cfg.dead_time = deads[rint_(0, 2)];
        cfg.max_events_per_ch = rint_(0, 1) ? 0 : (int)rint_(1, 5000);
        const int64_t rows_max = rint_(1, ((int64_t)1 << rint_(20, 31)) / N);
        cfg.max_chunk = rows_max * N;
        const bool fused = rint_(0, 1) == 1;
        Workspace ws;
        const char* e = size_workspace(cfg, fused, trig_slots, svf_lanes, kSvfW, ws);
        CHECK(e == nullptr, "size_workspace failed at max_chunk %lld: %s", (long long)cfg.max_chunk, e);
        if (e) continue;
        for (int call = 0; call < 8; ++call) {
            const int mode = call % 3;
            const int64_t rows = call < 3 ? rows_max : rint_(1, rows_max);
            std::vector<SubPlan> subs;
            int32_t stride = 0, capseg = 0;
            const char* pe = plan_call(ws, C, N, mode, cfg.dead_time, rows * N, subs, stride, capseg);
            CHECK(pe == nullptr, "legal call refused: %s (C %d rows %lld of %lld, mode %d, dead %d)", pe, C,
                  (long long)rows, (long long)rows_max, mode, cfg.dead_time);
            if (pe) continue;
            CHECK((int64_t)C * stride * capseg <= ws.slot_cap && capseg <= ws.scratch_cap, "tables");
        }
    }
}

// seg_capacity is a hard bound: the oracle trigger, driven to fire as often as it can, never puts
// more than seg_capacity(L, dead) packets of a channel into any window of L rows
static void fuzz_capacity(int iters) {
    for (int it = 0; it < iters; ++it) {
        const int C = (int)rint_(1, 8);
        const int64_t J = rint_(30, 3000);
        const int dead = (int)rint_(0, 40);
        const int mode = (int)rint_(0, 2);
        std::vector<int16_t> raw((size_t)(J * C)), taps((size_t)C * 26, 0), hist((size_t)25 * C, 0);
        std::vector<int32_t> thr(C), rearm(C);
        const int64_t q8 = rint_(0, 256);         // re-arm hysteresis (mkid_set_rearm)
        for (int c = 0; c < C; ++c) {
            taps[(size_t)c * 26] = 2047;          // identity matched filter: f = raw * 2047 >> 11
            thr[c] = (int32_t)rint_(-3000, 3000);
            rearm[c] = rearm_level(thr[c], (int32_t)q8);
        }
        const int kind = (int)rint_(0, 2);
        for (int64_t j = 0; j < J; ++j)
            for (int c = 0; c < C; ++c) {
                int v;
                if (kind == 0) v = (int)rint_(-32768, 32767);                         // noise
                else if (kind == 1) v = (j % 2) ? 20000 : -20000;                       // fastest cycling
                else v = (int)((j % (dead + 3)) == 0 ? -25000 : 25000) + (int)rint_(-50, 50);
                raw[(size_t)(j * C + c)] = (int16_t)v;
            }
        std::vector<trig_state> st(C);
        oracle_trig_reset_state(st.data(), C);
        const int64_t cap = J * C;
        std::vector<uint64_t> ev((size_t)cap);
        std::vector<int64_t> counts(C);
        const int64_t total = oracle_trigger(raw.data(), J, C, taps.data(), thr.data(), rearm.data(), mode, 41, 82, 93623,
                                             mode ? 8192 : 0, dead, hist.data(), st.data(), 0, ev.data(), cap,
                                             counts.data());
        CHECK(total <= cap, "trigger overflowed its own bound");
        // per channel: rows of its packets (ts = j - 1), every window of L rows
        std::vector<std::vector<int64_t>> rows(C);
        for (int64_t i = 0; i < std::min(total, cap); ++i) {
            const int c = (int)((ev[(size_t)i] >> MKID_PKT_CH_SHIFT) & 0xFFF);
            CHECK(c < C, "channel field");
            if (c < C) rows[c].push_back((int64_t)(ev[(size_t)i] & ((1ull << 28) - 1)));
        }
        for (int c = 0; c < C; ++c) {
            CHECK(counts[c] <= seg_capacity(J, dead), "whole-call bound: %lld > %lld", (long long)counts[c],
                  (long long)seg_capacity(J, dead));
            const std::vector<int64_t>& r = rows[c];
            CHECK(std::is_sorted(r.begin(), r.end()), "time order");
            for (int k = 0; k < 4 && !r.empty(); ++k) {
                const int64_t L = rint_(1, J);
                for (size_t a = 0; a < r.size(); ++a) {
                    const size_t b = std::upper_bound(r.begin(), r.end(), r[a] + L - 1) - r.begin();
                    CHECK((int64_t)(b - a) <= seg_capacity(L, dead), "window of %lld rows holds %lld > %lld",
                          (long long)L, (long long)(b - a), (long long)seg_capacity(L, dead));
                }
            }
        }
    }
}

static void fuzz_slot_order(int iters) {
    const int Cs[] = {64, 1024, 2048, 1024, 2048};
    for (int it = 0; it < iters; ++it) {
        const int C = Cs[rint_(0, 4)], N = 2 * C;
        std::vector<int32_t> bins(C);
        const int kind = (int)rint_(0, 2);
        for (int i = 0; i < C; ++i)
            bins[i] = kind == 0 ? (int32_t)rint_(0, N - 1) : (kind == 1 ? (int32_t)(i * 7 % N) : (int32_t)rint_(0, 3));
        std::vector<int16_t> so;
        slot_order(bins, C, so);
        std::vector<int> seen(C, 0);
        bool perm = (int)so.size() == C;
        for (int16_t v : so) perm = perm && v >= 0 && v < C && !seen[v]++;
        CHECK(perm, "slot order is not a permutation (C %d)", C);
        if (C == 1024 && perm)   // k_front3: wave w keeps channels 128 w .. 128 w + 127
            for (int slot = 0; slot < C; ++slot) {
                const int st = slot % (C / 2), w = st / 64;
                CHECK(so[slot] / 128 == w, "slot %d of wave %d holds channel %d", slot, w, so[slot]);
            }
        if (C == 2048 && perm)   // the k_front5 layout: each wave keeps the channels of its slots
            for (int slot = 0; slot < C; ++slot) {
                const int wave = slot < 1536 ? (slot % 512) / 64 : 8 + ((slot - 1536) % 256) / 64;
                const int ch = so[slot];
                const int cw = ch < 1536 ? (ch % 512) / 64 : 8 + ((ch - 1536) % 256) / 64;
                CHECK(cw == wave, "slot %d of wave %d holds channel %d", slot, wave, ch);
            }
    }
}

static void fuzz_quantize(int iters) {
    for (int it = 0; it < iters; ++it) {
        const int T = 4, N = (int)(1 << rint_(3, 12));
        std::vector<float> h((size_t)T * N);
        const int kind = (int)rint_(0, 3);
        const double scale = kind == 0 ? 1e-3 : (kind == 1 ? 1.0 : (kind == 2 ? 1e6 : 1e-30));
        for (float& v : h) v = (float)(std::uniform_real_distribution<double>(-1, 1)(rng) * scale);
        if (rint_(0, 5) == 0) std::fill(h.begin(), h.end(), 0.f);
        std::vector<int16_t> hq;
        const int S = quantize_pfb(h.data(), T, N, hq);
        CHECK((int)hq.size() == T * N && S >= -64 && S <= 64, "quantize geometry S %d", S);
        if (S > -64)
            for (int p = 0; p < N; ++p) {
                int64_t sp = 0;
                for (int t = 0; t < T; ++t) sp += std::abs((int64_t)hq[(size_t)t * N + p]);
                CHECK(sp <= 65535, "point %d tap sum %lld", p, (long long)sp);
            }
    }
}

static void fuzz_merge_pack(int iters) {
    for (int it = 0; it < iters; ++it) {
        const int C = (int)rint_(1, 300), nchunk = (int)rint_(1, 5);
        std::vector<uint64_t> ev;
        int64_t t0 = 0;
        for (int k = 0; k < nchunk; ++k) {   // each chunk channel-major, time-ascending
            for (int c = 0; c < C; ++c) {
                const int m = (int)rint_(0, 3);
                for (int i = 0; i < m; ++i)
                    ev.push_back(((uint64_t)c << MKID_PKT_CH_SHIFT) | ((uint64_t)rint_(0, 4095) << MKID_PKT_PEAK_SHIFT) |
                                 ((uint64_t)rint_(0, 4095) << MKID_PKT_BASE_SHIFT) | (uint64_t)(t0 + 10 * k + i));
            }
            t0 += 1000;
        }
        std::vector<uint64_t> m = ev;
        merge_channel_major(m.data(), (int64_t)m.size());
        bool ok = std::is_permutation(m.begin(), m.end(), ev.begin());
        for (size_t i = 1; i < m.size() && ok; ++i) {
            const uint64_t ca = m[i - 1] >> MKID_PKT_CH_SHIFT, cb = m[i] >> MKID_PKT_CH_SHIFT;
            ok = ca < cb || (ca == cb && (m[i - 1] & 0xFFFFFFF) < (m[i] & 0xFFFFFFF));
        }
        CHECK(ok, "merge is not channel-major / time-ascending");
        std::vector<uint64_t> out(m.size());
        const int r = pack_reference(m.data(), (int64_t)m.size(), out.data());
        uint64_t cmax = 0;
        for (uint64_t w : m) cmax = std::max<uint64_t>(cmax, w >> MKID_PKT_CH_SHIFT);
        CHECK((r == 0) == (m.empty() || cmax < 255), "pack_reference accepts exactly channels < 255 (max %llu, r %d)",
              (unsigned long long)cmax, r);
        if (r == 0)
            for (size_t i = 0; i < m.size(); ++i)
                CHECK((out[i] >> 56) == (m[i] >> MKID_PKT_CH_SHIFT) && (out[i] & 0xFFFFF) == (m[i] & 0xFFFFF),
                      "packed fields");
    }
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 300;
    rng.seed(argc > 2 ? strtoull(argv[2], nullptr, 10) : 12345);
    fuzz_plans(iters);
    fuzz_sizing(iters / 2 + 1);
    fuzz_capacity(iters / 3 + 1);
    fuzz_slot_order(iters / 10 + 2);
    fuzz_quantize(iters / 3 + 1);
    fuzz_merge_pack(iters);
    if (failures) {
        fprintf(stderr, "%d failures\n", failures);
        return 1;
    }
    printf("plan_fuzz ok: %d iterations\n", iters);
    return 0;
}
