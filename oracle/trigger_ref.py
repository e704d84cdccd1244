"""Pure-Python twin of oracle/trigger.c (small cases only) — TEST INFRASTRUCTURE.

Same semantics, written independently of the C so each pins the other (tests/test_oracle.py).
Reference anchors: see the header of oracle/trigger.c.
"""
import numpy as np

NT = 26
ARMED, PULSE, DEAD, REARM = 0, 1, 2, 3
HOLDOFF = 64      # start-of-stream hold-off (trigger.c HOLDOFF)


def trunc_div(n, d):
    q = abs(n) // abs(d)
    return q if (n >= 0) == (d > 0) else -q


def peakfit_i(y1, y2, y3):
    den = y3 + y1 - 2 * y2
    if den == 0:
        return y2
    return y2 - trunc_div((y3 - y1) ** 2, 8 * den)


def pack_wide(ch, peak, base, j):
    pk = min(max((peak >> 4) + 2048, 0), 4095)
    bs = min(max((base >> 4) + 2048, 0), 4095)
    return ((ch & 0xFFF) << 52) | (pk << 40) | (bs << 28) | (j & ((1 << 28) - 1))


def unpack_wide(w):
    w = int(w)
    return dict(ch=(w >> 52) & 0xFFF, peak=(w >> 40) & 0xFFF, base=(w >> 28) & 0xFFF,
                ts=w & ((1 << 28) - 1))


def new_state(C):
    return [dict(B=0, binit=0, st=DEAD, cnt=HOLDOFF, f1=0, f2=0, low=0, band=0) for _ in range(C)]


def trigger(raw, taps, thr, mode, alpha, kf, kq, base_thr, dead, hist=None, state=None, j0=0, rearm=None):
    """raw [J][C] int; taps [C][26]; rearm [C] re-arm levels (None: the thresholds); returns
    (events list channel-major, hist, state)."""
    rearm = thr if rearm is None else rearm
    raw = np.asarray(raw, np.int64)
    J, C = raw.shape
    hist = np.zeros((25, C), np.int64) if hist is None else np.asarray(hist, np.int64).copy()
    state = new_state(C) if state is None else [dict(s) for s in state]
    full = np.concatenate([hist, raw])          # full[25 + j] = raw_j
    events = []
    for c in range(C):
        s = state[c]
        a = [int(t) for t in taps[c]]
        col = [int(v) for v in full[:, c]]
        for j in range(J):
            acc = 0
            for i in range(NT):
                acc += a[i] * col[25 + j - i]
            f = min(max(acc >> 11, -32768), 32767)
            if not s['binit'] and s['st'] != DEAD:
                s['B'] = 0 if mode == 0 else f
                s['low'] = f << 16
                s['band'] = 0
                s['binit'] = 1
            base_prev = (s['low'] >> 16) if mode == 2 else s['B']
            e = f - base_prev
            gate = base_thr <= 0 or (-base_thr < e < base_thr)
            if s['binit'] and mode == 1 and gate:
                s['B'] += (alpha * e) >> 9
            elif s['binit'] and mode == 2 and gate:
                high = (f << 16) - s['low'] - ((kq * s['band']) >> 16)
                s['band'] += (kf * high) >> 16
                s['low'] += (kf * s['band']) >> 16
            if s['st'] == ARMED:
                if e < thr[c]:
                    s['st'] = PULSE
            elif s['st'] == PULSE:
                if f > s['f1']:
                    pk = peakfit_i(s['f2'], s['f1'], f)
                    events.append(pack_wide(c, pk, base_prev, j0 + j - 1))
                    s['st'] = DEAD
                    s['cnt'] = dead
            elif s['st'] == DEAD:
                s['cnt'] -= 1
                if s['cnt'] <= 0:
                    s['st'] = REARM
            else:
                if e >= rearm[c]:
                    s['st'] = ARMED
            s['f2'] = s['f1']
            s['f1'] = f
    new_hist = full[len(full) - 25:].copy()
    return events, new_hist, state
