"""Python front-end of one MI355X channeliser context (one feedline on one GPU).

This is the host-side mirror of the firmware configuration the reference performs over katcp
(ROACH_Setup.py / ROACH_Pulses.py) — every setter maps to one register group (see
include/mkidgpu.h) — and of its data path: ``process`` runs the HIP kernels (PFB+FFT+DDC, IQ
low-pass + phase, matched-filter trigger) and returns the phase stream and photon packets.
"""
import ctypes

import numpy as np

from . import _lib
from .pfb import pfb_prototype


def _ptr(a):
    """Host numpy array / torch tensor / int -> void*."""
    if a is None:
        return None
    if isinstance(a, int):
        return ctypes.c_void_p(a)
    if hasattr(a, 'data_ptr'):
        return ctypes.c_void_p(a.data_ptr())
    return a.ctypes.data_as(ctypes.c_void_p)


class Channelizer:
    def __init__(self, n_channels, device=0, max_chunk=1 << 22, dead_time=32, sample_rate=512e6,
                 max_events_per_ch=0, lib_path=None, front='auto'):
        self._L = _lib.load(lib_path)
        cfg = _lib.Cfg()
        _lib.check(self._L.mkid_default_cfg(ctypes.byref(cfg), int(n_channels)))
        cfg.max_chunk = int(max_chunk)
        cfg.dead_time = int(dead_time)
        cfg.sample_rate = float(sample_rate)
        cfg.max_events_per_ch = int(max_events_per_ch)
        if front not in ('auto', 'split'):
            raise ValueError("front must be 'auto' (fused K1-K6 where supported) or 'split'")
        cfg.front = _lib.FRONT_AUTO if front == 'auto' else _lib.FRONT_SPLIT
        h = ctypes.c_void_p()
        _lib.check(self._L.mkid_create(ctypes.byref(cfg), int(device), ctypes.byref(h)))
        self._h = h
        self.cfg = cfg
        self.device = int(device)
        self.C = cfg.n_channels
        self.N = cfg.fft_len
        self.P = cfg.dds_entries
        self.set_pfb(pfb_prototype(self.N, cfg.pfb_taps))

    # ---- lifecycle -------------------------------------------------------------------------
    def torch_device(self):
        """The torch device of this context's GPU (allocations for it go there, not to the
        current device)."""
        import torch
        return torch.device('cuda', self.device)

    def close(self):
        if getattr(self, '_h', None):
            self._L.mkid_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc):
        if rc != _lib.MKID_OK:
            msg = (self._L.mkid_last_error(self._h) or b'').decode(errors='replace')
            raise _lib.MkidError(rc, msg)
        return rc

    # ---- configuration (one register group each) ---------------------------------------------
    def set_stream(self, stream_ptr):
        """Run on an external hipStream_t (e.g. a torch.cuda.Stream's cuda_stream); 0/None
        restores the context's own non-blocking stream. torch's default stream has handle 0, so
        to share a stream with torch work use a torch.cuda.Stream, not the default one."""
        self._chk(self._L.mkid_set_stream(self._h, ctypes.c_void_p(stream_ptr or 0)))

    def set_pfb(self, coeffs):
        c = np.ascontiguousarray(coeffs, np.float32)
        self._chk(self._L.mkid_set_pfb(self._h, _ptr(c), c.size))

    def set_bins(self, bins):
        b = np.ascontiguousarray(bins, np.int32)
        self._chk(self._L.mkid_set_bins(self._h, _ptr(b), b.size))

    def set_dds(self, lut_i, lut_q):
        li = np.ascontiguousarray(lut_i, np.int16).reshape(self.C, -1)
        lq = np.ascontiguousarray(lut_q, np.int16).reshape(self.C, -1)
        self._chk(self._L.mkid_set_dds(self._h, _ptr(li), _ptr(lq), li.shape[1]))

    def set_lpf(self, taps12):
        t = np.ascontiguousarray(taps12, np.int16)
        self._chk(self._L.mkid_set_lpf(self._h, _ptr(t), t.size))

    def set_fir(self, taps12):
        t = np.ascontiguousarray(taps12, np.int16).reshape(self.C, -1)
        self._chk(self._L.mkid_set_fir(self._h, _ptr(t), t.shape[0], t.shape[1]))

    def set_centers(self, ic, qc):
        i = np.ascontiguousarray(ic, np.float32)
        q = np.ascontiguousarray(qc, np.float32)
        self._chk(self._L.mkid_set_centers(self._h, _ptr(i), _ptr(q), i.size))

    def set_thresholds(self, thr):
        t = np.ascontiguousarray(thr, np.int32)
        self._chk(self._L.mkid_set_thresholds(self._h, _ptr(t), t.size))

    def set_baseline(self, mode=_lib.BASE_EMA, alpha=41, kf=82, kq=93623, base_thr=8192):
        self._chk(self._L.mkid_set_baseline(self._h, int(mode), int(alpha), int(kf), int(kq),
                                            int(base_thr)))

    def set_rearm(self, frac_q8):
        """Trigger re-arm hysteresis (mkid_set_rearm): re-arm at thr - floor(thr * frac_q8 / 256)."""
        self._chk(self._L.mkid_set_rearm(self._h, int(frac_q8)))

    def reset(self):
        self._chk(self._L.mkid_reset_stream(self._h))

    # ---- data path ---------------------------------------------------------------------------
    def process(self, iq, want_phase=True, cap=None):
        """iq: int16 [S][2] host array. Returns (phase [S/N][C] float32 or None, events uint64)."""
        x = np.ascontiguousarray(iq, np.int16).reshape(-1, 2)
        S = x.shape[0]
        J = S // self.N
        phase = np.empty((J, self.C), np.float32) if want_phase else None
        cap = J * self.C if cap is None else int(cap)
        ev = np.empty(max(cap, 1), np.uint64)
        n = ctypes.c_int64()
        rc = self._L.mkid_process(self._h, _ptr(x), S, _ptr(phase), _ptr(ev), cap, ctypes.byref(n))
        self._chk(rc)
        return phase, ev[:n.value].copy()

    def process_device(self, d_iq, nsamples, d_phase, d_events, cap, d_counts):
        """Device pointers (ints or torch tensors); asynchronous on the context stream."""
        self._chk(self._L.mkid_process_device(self._h, _ptr(d_iq), int(nsamples), _ptr(d_phase),
                                              _ptr(d_events), int(cap), _ptr(d_counts)))

    def trigger_phase_device(self, d_raw, rows, d_events, cap, d_counts):
        """K7 + K8 on device Fix16_13 phase rows [rows][C] (mkid_trigger_phase)."""
        self._chk(self._L.mkid_trigger_phase(self._h, _ptr(d_raw), int(rows), _ptr(d_events), int(cap),
                                             _ptr(d_counts)))

    def trigger_phase(self, raw):
        """Host convenience: raw int16 [rows][C] -> packets (uint64, channel-major)."""
        import torch
        dev = self.torch_device()
        r = np.ascontiguousarray(raw, np.int16).reshape(-1, self.C)
        d_raw = torch.from_numpy(r).to(dev)
        cap = r.shape[0] * self.C // 2 + 64
        d_ev = torch.empty(cap, dtype=torch.int64, device=dev)
        d_cnt = torch.zeros(2, dtype=torch.int64, device=dev)
        torch.cuda.synchronize(dev)
        self.trigger_phase_device(d_raw, r.shape[0], d_ev, cap, d_cnt)
        torch.cuda.synchronize(dev)
        n = d_cnt.cpu().numpy()
        if n[0] > n[1]:
            raise _lib.MkidError(_lib.MKID_E_OVERFLOW, 'trigger_phase: packets dropped')
        return d_ev[:int(n[1])].cpu().numpy().view(np.uint64).copy()

    def raw_phase_ptr(self):
        p = ctypes.c_void_p()
        n = ctypes.c_int64()
        self._chk(self._L.mkid_last_raw_phase(self._h, ctypes.byref(p), ctypes.byref(n)))
        return p.value, n.value

    def raw_phase(self):
        """Host copy of the last sub-chunk's Fix16_13 phase rows, int16 [rows][C]."""
        p, rows = self.raw_phase_ptr()
        out = np.empty((rows, self.C), np.int16)
        n = ctypes.c_int64()
        self._chk(self._L.mkid_read_raw_phase(self._h, _ptr(out), rows, ctypes.byref(n)))
        return out

    def set_iq_tap(self, channel):
        """Record channel's low-pass output (IQ snapshot source); channel < 0 turns it off."""
        self._chk(self._L.mkid_set_iq_tap(self._h, int(channel)))

    def iq_tap(self):
        """int16 [rows][2] I/Q of the tapped channel for the rows of the last process call."""
        n = ctypes.c_int64()
        self._chk(self._L.mkid_read_iq_tap(self._h, None, 0, ctypes.byref(n)))
        out = np.empty((n.value, 2), np.int16)
        self._chk(self._L.mkid_read_iq_tap(self._h, _ptr(out), n.value, ctypes.byref(n)))
        return out

    def trigger_reruns(self):
        n = ctypes.c_int64()
        self._chk(self._L.mkid_trigger_reruns(self._h, ctypes.byref(n)))
        return n.value

    def set_accumulator(self, on):
        """startAccumulator (ROACH_Setup.py:654-659): True arms the avgIQ accumulator (the sums
        restart; every following process call adds its rows), False stops it (sums kept)."""
        self._chk(self._L.mkid_set_accumulator(self._h, 1 if on else 0))

    def avg_iq(self):
        """Per-channel mean low-pass I/Q over the rows accumulated since set_accumulator(True)."""
        mi = np.empty(self.C, np.float32)
        mq = np.empty(self.C, np.float32)
        self._chk(self._L.mkid_avg_iq(self._h, _ptr(mi), _ptr(mq)))
        return mi, mq

    # ---- host-replay triggers --------------------------------------------
    def replay_trigger(self, d_raw, n, ld, nch, mode, length, start, need, skip, threshold_deg,
                       wrap_negative=False, d_hits=None, cap=64, d_counts=None):
        """Run the reference's rolling-/block-mean replay trigger on device Fix16_13 phase
        d_raw[n][ld] (int16 device tensor or pointer), channels 0..nch-1. Returns the device
        (hits [nch, cap] int32, counts [nch] int32) tensors (allocated when not given)."""
        import torch
        if d_hits is None:
            d_hits = torch.full((nch, cap), -1, dtype=torch.int32, device=self.torch_device())
        if d_counts is None:
            d_counts = torch.zeros(nch, dtype=torch.int32, device=self.torch_device())
        rc = _lib.ReplayCfg(int(mode), int(length), int(start), int(need), int(skip),
                            1 if wrap_negative else 0, float(threshold_deg))
        self._chk(self._L.mkid_replay_trigger(self._h, _ptr(d_raw), int(n), int(ld), int(nch),
                                              ctypes.byref(rc), _ptr(d_hits), int(cap), _ptr(d_counts)))
        return d_hits, d_counts

    # ---- per-packet optimal-filter pulse height (BASELINE config 5) -----------------------------
    def set_pulse_filter(self, coeff, pre):
        """coeff: float [C][ncoeff] (one filter per channel, e.g. template.optimal_filter's weights
        tiled); the height of a packet stamped ts is sum_i coeff[ch][i] phase[ts - pre + i][ch]."""
        cf = np.ascontiguousarray(coeff, np.float32).reshape(self.C, -1)
        self._chk(self._L.mkid_set_pulse_filter(self._h, _ptr(cf), cf.shape[0], cf.shape[1], int(pre)))

    def pulse_heights_device(self, d_phase, rows, j0, d_events, n, d_heights):
        """Device pointers; asynchronous on the context stream (include/mkidgpu.h)."""
        self._chk(self._L.mkid_pulse_heights(self._h, _ptr(d_phase), int(rows), int(j0), _ptr(d_events),
                                             int(n), _ptr(d_heights)))

    def pulse_heights_counted(self, d_phase, rows, j0, d_events, d_count, cap, d_heights):
        """As pulse_heights_device with the packet count read on the device (d_count: an int64
        device pointer/tensor, e.g. the d_counts[1:] of the process call)."""
        self._chk(self._L.mkid_pulse_heights_counted(self._h, _ptr(d_phase), int(rows), int(j0), _ptr(d_events),
                                                     _ptr(d_count), int(cap), _ptr(d_heights)))

    def pulse_heights(self, phase, events, j0=0):
        """Host convenience: phase float32 [rows][C] (rad) of global rows j0.., events uint64 [n]
        -> float32 heights [n] (NaN where the window leaves the rows)."""
        import torch
        dev = self.torch_device()
        ph = torch.from_numpy(np.ascontiguousarray(phase, np.float32)).to(dev)
        ev = torch.from_numpy(np.ascontiguousarray(events, np.uint64).view(np.int64)).to(dev)
        out = torch.empty(ev.numel(), dtype=torch.float32, device=dev)
        torch.cuda.synchronize(dev)  # the uploads run on torch's stream, the kernel on the context's
        self.pulse_heights_device(ph, ph.shape[0], j0, ev, ev.numel(), out)
        torch.cuda.synchronize(dev)
        return out.cpu().numpy()

    # ---- timing ------------------------------------------------------------------------------
    def set_timing(self, on, kernels=None):
        """on: time every kernel (HIP events); kernels: names (e.g. ['k_front']) to time only
        those (mkid_set_timing with MKID_TIMING_ONLY masks; each timed launch costs two event
        records on the stream)."""
        if on and kernels:
            names = [self._L.mkid_kernel_name(k).decode() for k in range(_lib.K_COUNT)]
            mask = 0
            for n in kernels:
                if n not in names:
                    raise ValueError('unknown kernel %r (one of %s)' % (n, names))
                mask |= 1 << names.index(n)
            self._chk(self._L.mkid_set_timing_mask(self._h, mask))
        else:
            self._chk(self._L.mkid_set_timing(self._h, 1 if on else 0))

    def timing(self):
        out = {}
        for k in range(_lib.K_COUNT):
            ms = ctypes.c_double()
            n = ctypes.c_int64()
            self._chk(self._L.mkid_get_timing(self._h, k, ctypes.byref(ms), ctypes.byref(n)))
            out[self._L.mkid_kernel_name(k).decode()] = (ms.value, n.value)
        return out

    def stream_copy(self, d_dst, d_src, nbytes):
        """Diagnostic HBM copy (mkid_stream_copy), asynchronous on the context stream."""
        self._chk(self._L.mkid_stream_copy(self._h, _ptr(d_dst), _ptr(d_src), int(nbytes)))

    # ---- synthetic source (tests / bench only) -------------------------------------------------
    def synth_adc(self, d_out, nsamples, n0, d_base, d_tones, d_pulses, npulses, tau_rise,
                  tau_fall, window, sigma, seed):
        self._chk(self._L.mkid_synth_adc(self._h, _ptr(d_out), int(nsamples), int(n0),
                                         _ptr(d_base), _ptr(d_tones), _ptr(d_pulses),
                                         int(npulses), float(tau_rise), float(tau_fall),
                                         int(window), float(sigma), int(seed) & 0xffffffff))


def pack_reference(wide):
    """Wide device packets -> reference 64-bit packets (mkid_pack_reference, C <= 254)."""
    L = _lib.load()
    w = np.ascontiguousarray(wide, np.uint64)
    out = np.empty_like(w)
    _lib.check(L.mkid_pack_reference(_ptr(w), w.size, _ptr(out)))
    return out
