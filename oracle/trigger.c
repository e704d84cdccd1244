/* C restatement of the trigger stages K7/K8 — TEST INFRASTRUCTURE (see oracle/__init__.py).
 *
 * Pinned values from the reference: matched-filter taps are the 12-bit int(lpf*(2**11-1))
 * quantisation of ROACH_Pulses.py:69,88-92 (CUSTOM_FIR=matched_30us.txt, setEnvironment.sh:34);
 * thresholds are Fix16_13 relative to the baseline and negative-going (ROACH_Pulses.py:270);
 * EMA alpha Fix12_9 (set_alpha.py:10-11 -> 41), SVF Kf/Kq Fix18_16 (set_svf.py:33-44 -> 82,
 * 93623), baseline gate Fix16_13 (set_base_thresh.py:9-10 -> 8192); peak = 3-point parabolic fit
 * (Utils/bin.py:12-16) in integer arithmetic; packet fields Fix12_9 offset-binary
 * (ROACH_Pulses.py:852-859, Utils/bin.py:5-7). The state machine (edge trigger, peak on the first
 * upturn, dead time, re-arm at the re-arm level) is a build decision: the firmware is absent.
 * Re-arm level (round 5, hysteresis): a channel re-arms after its dead time once e >= rearm[c];
 * rearm = thr (NULL) is the round-1..4 rule. mkid_set_rearm derives the levels from the thresholds
 * (oracle/trigger.py rearm_levels); the reference's own host replay re-arms only after a fixed
 * 1000-sample skip (pulse_triggering_v2.py:104-174).
 *
 * Semantics shared bit-for-bit with mkids_sdr_amd/csrc/k_trigger.hip and oracle/trigger_ref.py.
 */
#include <stdint.h>
#include <string.h>

#define NT 26
enum { ST_ARMED = 0, ST_PULSE = 1, ST_DEAD = 2, ST_REARM = 3 };
/* Start-of-stream hold-off (build decision): after a reset the trigger state is
 * DEAD for HOLDOFF samples with no baseline, so the filters' start-up transient (zero PFB / low-pass
 * / matched-filter history) neither fires the trigger nor seeds the baseline; the baseline is
 * initialised from the first sample after it. */
#define HOLDOFF 64

typedef struct {
    int32_t B, binit, st, cnt, f1, f2, pad0, pad1;
    int64_t low, band;
} trig_state; /* 48 bytes, identical layout to the device struct */

int32_t oracle_trig_state_size(void) { return (int32_t)sizeof(trig_state); }

static inline int32_t clamp16(int32_t v) { return v < -32768 ? -32768 : (v > 32767 ? 32767 : v); }
static inline int32_t clampi(int32_t v, int32_t lo, int32_t hi) { return v < lo ? lo : (v > hi ? hi : v); }

int64_t peakfit_i(int64_t y1, int64_t y2, int64_t y3) {
    int64_t den = y3 + y1 - 2 * y2;
    if (den == 0) return y2;
    int64_t d = y3 - y1;
    return y2 - (d * d) / (8 * den); /* C division truncates toward zero */
}

uint64_t pack_wide(int32_t ch, int64_t peak, int32_t base, int64_t j) {
    uint64_t pk = (uint64_t)clampi((int32_t)((peak >> 4) + 2048), 0, 4095);
    uint64_t bs = (uint64_t)clampi((base >> 4) + 2048, 0, 4095);
    return ((uint64_t)(ch & 0xFFF) << 52) | (pk << 40) | (bs << 28) | ((uint64_t)j & ((1ull << 28) - 1));
}

/* State of a freshly reset channel: hold-off, no baseline yet. */
void oracle_trig_reset_state(trig_state* st, int32_t C) {
    memset(st, 0, sizeof(trig_state) * (size_t)C);
    for (int32_t c = 0; c < C; ++c) {
        st[c].st = ST_DEAD;
        st[c].cnt = HOLDOFF;
    }
}

/* raw: [J][C] int16 Fix16_13 time-major; hist: [25][C] previous raw (hist[24] = newest);
 * taps: [C][26] int12; st: [C]; rearm: [C] re-arm levels or NULL (= thr). Events are written channel-major, time-ascending; returns the
 * total number produced (may exceed cap; only cap are written). counts[c] (nullable) = per-ch. */
int64_t oracle_trigger(const int16_t* raw, int64_t J, int32_t C, const int16_t* taps,
                       const int32_t* thr, const int32_t* rearm, int32_t mode, int32_t alpha, int32_t kf, int32_t kq,
                       int32_t base_thr, int32_t dead, int16_t* hist, trig_state* st, int64_t j0,
                       uint64_t* ev, int64_t cap, int64_t* counts) {
    int64_t total = 0;
    for (int32_t c = 0; c < C; ++c) {
        trig_state s = st[c];
        const int32_t lvl = rearm ? rearm[c] : thr[c];
        int64_t nc = 0;
        for (int64_t j = 0; j < J; ++j) {
            int32_t acc = 0;
            for (int i = 0; i < NT; ++i) {
                int64_t jj = j - i;
                int32_t r = jj >= 0 ? raw[jj * C + c] : hist[(25 + jj) * C + c];
                acc += (int32_t)taps[c * NT + i] * r;
            }
            int32_t f = clamp16(acc >> 11);
            if (!s.binit && s.st != ST_DEAD) { /* first sample after the hold-off */
                s.B = (mode == 0) ? 0 : f;
                s.low = (int64_t)f * 65536;
                s.band = 0;
                s.binit = 1;
            }
            int32_t base_prev = (mode == 2) ? (int32_t)(s.low >> 16) : s.B;
            int32_t e = f - base_prev;
            int gate = (base_thr <= 0) || (e < base_thr && e > -base_thr);
            if (s.binit && mode == 1 && gate) {
                s.B += (alpha * e) >> 9;
            } else if (s.binit && mode == 2 && gate) {
                int64_t high = ((int64_t)f * 65536) - s.low - (((int64_t)kq * s.band) >> 16);
                s.band += ((int64_t)kf * high) >> 16;
                s.low += ((int64_t)kf * s.band) >> 16;
            }
            switch (s.st) {
                case ST_ARMED:
                    if (e < thr[c]) s.st = ST_PULSE;
                    break;
                case ST_PULSE:
                    if (f > s.f1) {
                        int64_t pk = peakfit_i(s.f2, s.f1, f);
                        if (total < cap) ev[total] = pack_wide(c, pk, base_prev, j0 + j - 1);
                        ++total;
                        ++nc;
                        s.st = ST_DEAD;
                        s.cnt = dead;
                    }
                    break;
                case ST_DEAD:
                    s.cnt -= 1;
                    if (s.cnt <= 0) s.st = ST_REARM;
                    break;
                default:
                    if (e >= lvl) s.st = ST_ARMED;
                    break;
            }
            s.f2 = s.f1;
            s.f1 = f;
        }
        /* roll the 25-sample history */
        for (int i = 0; i < 25; ++i) {
            int64_t jj = J - 25 + i;
            int16_t v = jj >= 0 ? raw[jj * C + c] : hist[(25 + jj) * C + c];
            hist[i * C + c] = v; /* safe: reads of hist at index 25+jj > i*C+c row only when jj<0 */
        }
        st[c] = s;
        if (counts) counts[c] = nc;
    }
    return total;
}
