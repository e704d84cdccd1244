"""ctypes front-end of oracle/trigger.c — TEST INFRASTRUCTURE (see oracle/__init__.py)."""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, '_build', 'liboracle.so')
_lib = None

STATE_DTYPE = np.dtype([('B', '<i4'), ('binit', '<i4'), ('st', '<i4'), ('cnt', '<i4'),
                        ('f1', '<i4'), ('f2', '<i4'), ('pad0', '<i4'), ('pad1', '<i4'),
                        ('low', '<i8'), ('band', '<i8')])


def build():
    """Compile oracle/trigger.c with gcc (make -C oracle)."""
    subprocess.check_call(['make', '-s', '-C', _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        P = ctypes.c_void_p
        L.oracle_trigger.restype = ctypes.c_int64
        L.oracle_trigger.argtypes = [P, ctypes.c_int64, ctypes.c_int32, P, P, P, ctypes.c_int32,
                                     ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                     ctypes.c_int32, ctypes.c_int32, P, P, ctypes.c_int64, P,
                                     ctypes.c_int64, P]
        L.oracle_trig_state_size.restype = ctypes.c_int32
        L.oracle_trig_reset_state.restype = None
        L.oracle_trig_reset_state.argtypes = [P, ctypes.c_int32]
        assert L.oracle_trig_state_size() == STATE_DTYPE.itemsize
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def rearm_levels(thr, frac_q8):
    """Re-arm level per channel for a hysteresis fraction frac_q8 / 256 (mkid_set_rearm): the level
    moves from the threshold toward 0 (the baseline): lvl = thr - floor(thr * frac_q8 / 256).
    frac_q8 = 0 gives lvl = thr (the round-1..4 rule)."""
    t = np.asarray(thr, np.int64)
    return (t - ((t * int(frac_q8)) >> 8)).astype(np.int32)


class Trigger:
    """Streaming trigger over [J][C] int16 raw phase."""

    def __init__(self, C, taps, thr, mode=1, alpha=41, kf=82, kq=93623, base_thr=8192,
                 dead=32, rearm_q8=0):
        self.C = C
        self.taps = np.ascontiguousarray(taps, np.int16).reshape(C, 26)
        self.thr = np.ascontiguousarray(thr, np.int32).reshape(C)
        self.rearm = np.ascontiguousarray(rearm_levels(self.thr, rearm_q8), np.int32)
        self.params = (mode, alpha, kf, kq, base_thr, dead)
        self.reset()

    def reset(self):
        self.hist = np.zeros((25, self.C), np.int16)
        self.state = np.zeros(self.C, STATE_DTYPE)
        lib().oracle_trig_reset_state(_p(self.state), self.C)   # start-of-stream hold-off
        self.j0 = 0

    def run(self, raw, cap=None):
        raw = np.ascontiguousarray(raw, np.int16)
        J = raw.shape[0]
        cap = J * self.C if cap is None else cap
        ev = np.zeros(max(cap, 1), np.uint64)
        counts = np.zeros(self.C, np.int64)
        mode, alpha, kf, kq, bt, dead = self.params
        n = lib().oracle_trigger(_p(raw), J, self.C, _p(self.taps), _p(self.thr), _p(self.rearm), mode, alpha, kf,
                                 kq, bt, dead, _p(self.hist), _p(self.state), self.j0, _p(ev), cap,
                                 _p(counts))
        self.j0 += J
        return ev[:min(n, cap)].copy(), int(n), counts
