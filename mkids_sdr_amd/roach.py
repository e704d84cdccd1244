"""FpgaClient-compatible register shim + the ChannelizerControls setup surface, over the GPU.

The reference drives its firmware with ``corr.katcp_wrapper.FpgaClient(ip, 7147)`` and five calls
(ROACH_Setup.py:112-115, 545-547, 570, 603-605, 659, 887; ROACH_Pulses.py:95-97, 242-248,
286-288, 796-800): ``progdev``, ``write_int``, ``write``, ``read``, ``read_int``. ``FpgaClient``
below accepts exactly those calls and register names, decodes every configuration write into
the device configuration of one MI355X channeliser context (include/mkidgpu.h), and serves the
readback registers from the GPU's outputs on a DAC->ADC loop-back source (the conjugated DAC LUT,
ROACH_Setup.py:485-487). ``RoachSetup`` / ``RoachPulses`` restate the reference's AppForm methods
(same names and argument meaning, GUI widgets replaced by attributes) on top of it, so
ChannelizerControls-style code runs unchanged against the GPU.

Register map:
  config   bins/load_bins, dram_memory, FIR_b{2n}b{2n+1}/FIR_load_coeff, capture_threshold/
           capture_load_thresh, conv_phase_centers/conv_phase_load_centers,
           capture_Baseline_alpha, capture_base_Kf, capture_base_Kq, capture_base_thresh
  control  startDAC, DRAM_LUT_rd_valid, startAccumulator, avgIQ_ctrl, startSnap, snapPhase_ctrl,
           ch_we, startBuffer, conv_phase_startSnap{I,Q,IQ,Phase} / conv_phase_snap{...}_ctrl
  readback avgIQ_bram, snapPhase_bram (ROACH_Pulses.py snapshot, swapped halves), qdr0_memory
           (longsnapshot, ROACH_Pulses.py:433-551), conv_phase_snapPhase_bram /
           conv_phase_snapIQ_bram / conv_phase_snapI_bram / conv_phase_snapQ_bram with
           conv_phase_ch_we_Phase / conv_phase_ch_we_IQ, one shared capture per startSnap strobe
           (pulse_triggering_v2.py:36-95, pulse_triggering_IQ.py:36-147, ROACH_Pulses_IQ.py:357-407,
           readouttesterIQ.py:34-88), pulses_addr, pulses_bram0/1
Errors are raised as RuntimeError (katcp semantics, pulse_triggering_v2.py:177-179).
"""
import re
import struct

import numpy as np

from . import codecs, replay, lut, packets

FIR_RE = re.compile(r'^FIR_b(\d+)b(\d+)$')
PULSE_RING = 2 ** 14          # pulses_bram0/1 depth (ROACH_Pulses.py:799-800)
# conv_phase snapshot BRAMs: bytes per phase row in the read (one '>h' sample per 32-bit word at
# bytes [2:4] for I, Q and phase, readouttesterIQ.py:71-74; 16 bytes per 2 rows for the packed IQ
# BRAM, pulse_triggering_IQ.py:121-147) and the startSnap strobe that arms each
SNAP_ROW_BYTES = {'conv_phase_snapI_bram': 4, 'conv_phase_snapQ_bram': 4,
                  'conv_phase_snapPhase_bram': 4, 'conv_phase_snapIQ_bram': 8}
SNAP_STROBES = {'conv_phase_startSnapI': 'conv_phase_snapI_bram',
                'conv_phase_startSnapQ': 'conv_phase_snapQ_bram',
                'conv_phase_startSnapPhase': 'conv_phase_snapPhase_bram',
                'conv_phase_startSnapIQ': 'conv_phase_snapIQ_bram'}


class DeviceConfig:
    """Decoded firmware configuration (pure host state; pushed to a Channelizer by sync())."""

    def __init__(self, n_channels, dds_lag=lut.DDS_LAG):
        C = n_channels
        self.C = C
        self.dds_lag = dds_lag
        self.bins = np.arange(C, dtype=np.int64)
        self.lut_i = np.full((C, lut.LUT_LEN // C), 32767, np.int64)
        self.lut_q = np.zeros((C, lut.LUT_LEN // C), np.int64)
        self.dac_i = np.zeros(lut.LUT_LEN, np.int64)
        self.dac_q = np.zeros(lut.LUT_LEN, np.int64)
        self.fir = np.zeros((C, 26), np.int64)
        self.thr = np.full(C, -(1 << 30), np.int64)
        self.ic = np.zeros(C, np.float32)
        self.qc = np.zeros(C, np.float32)
        self.baseline = dict(mode=1, alpha=41, kf=82, kq=93623, base_thr=8192)
        self.dirty = set(['bins', 'dds', 'fir', 'thr', 'centers', 'baseline'])


class FpgaClient:
    """katcp FpgaClient look-alike over one GPU channeliser context."""

    def __init__(self, host='mi355x', port=7147, n_channels=256, device=0, sample_rate=512e6,
                 dds_lag=lut.DDS_LAG, gpu=True, noise_sigma=0.0, seed=0):
        self.host, self.port = host, port
        self.C = n_channels
        self.N = 2 * n_channels
        self.fs = sample_rate
        self.device = device
        self.regs = {}
        self.cfg = DeviceConfig(n_channels, dds_lag)
        self.gpu = gpu
        self.noise_sigma = noise_sigma
        self.rng = np.random.default_rng(seed)
        self._chan = None
        self._t = 0                      # loop-back source position (ADC samples)
        self._j = 0                      # phase rows the device stream has processed since reset
        # photon-packet wire path (packets.py): time-ordered words with us-since-PPS stamps and
        # end-of-second markers into the pulses_bram0/1 ring while startBuffer is 1
        self._wire = packets.WireStream(sample_rate, self.N)
        self.ring = packets.PulseRing()
        self._buffering = False
        self.pulse_rows = 4096           # phase rows streamed between two pulses_addr reads
        self.packet_log = None           # a list to record (wide packets, j0, rows) per call
        self.lo = None                   # current LO (set_lo); None = nominal
        self.lo_nominal = None
        self.resonators = []             # RESDIFF parameter dicts (set_resonators)
        self._adc_cache = None
        self.boffile = None
        self._armed = set()              # conv_phase snapshot BRAMs armed by a startSnap strobe
        self._snaps = {}                 # BRAM -> the capture it holds

    # ---- katcp surface -----------------------------------------------------------------------
    def progdev(self, boffile):
        self.boffile = boffile
        self.regs.clear()
        self.cfg = DeviceConfig(self.C, self.cfg.dds_lag)
        self._t = 0
        if self._chan is not None:
            self._chan.reset()
        self._j = 0
        self._wire = packets.WireStream(self.fs, self.N)
        self.ring = packets.PulseRing()
        self._adc_cache = None
        self._armed, self._snaps = set(), {}
        return 'ok'

    def is_connected(self):
        return True

    def listdev(self):
        return sorted(self.regs)

    def write_int(self, name, value, blindwrite=False, offset=0):
        value = int(value)
        prev = self.regs.get(name, 0)
        self.regs[name] = value
        rising = (value & 1) and not (prev & 1)
        if name == 'load_bins' and rising:
            self.cfg.bins[value >> 1] = self.regs.get('bins', 0) % self.N
            self.cfg.dirty.add('bins')
        elif name == 'FIR_load_coeff' and rising:
            ch = value >> 1
            for n in range(13):
                key = 'FIR_b%db%d' % (2 * n, 2 * n + 1)
                if key in self.regs:
                    self.cfg.fir[ch, 2 * n], self.cfg.fir[ch, 2 * n + 1] = \
                        codecs.decode_fir_register(self.regs[key])
            self.cfg.dirty.add('fir')
        elif name == 'capture_load_thresh' and rising:
            self.cfg.thr[value >> 1] = _s32(self.regs.get('capture_threshold', 0))
            self.cfg.dirty.add('thr')
        elif name == 'conv_phase_load_centers' and rising:
            ic, qc = codecs.decode_center_register(_s32(self.regs.get('conv_phase_centers', 0)))
            ch = value >> 1
            self.cfg.ic[ch], self.cfg.qc[ch] = ic, qc
            self.cfg.dirty.add('centers')
        elif name in ('capture_Baseline_alpha', 'capture_base_Kf', 'capture_base_Kq',
                      'capture_base_thresh', 'capture_base_mode'):
            key = dict(capture_Baseline_alpha='alpha', capture_base_Kf='kf', capture_base_Kq='kq',
                       capture_base_thresh='base_thr', capture_base_mode='mode')[name]
            self.cfg.baseline[key] = value
            self.cfg.dirty.add('baseline')
        elif name == 'startBuffer':
            self.ring.start_buffer(value & 1, prev & 1)
            self._buffering = bool(value & 1)
        elif name == 'conv_phase_ch_we_IQ' and self._chan is not None:
            self._chan.set_iq_tap(value)
        elif name in SNAP_STROBES:
            # conv_phase_startSnap{I,Q,IQ,Phase} 0 -> 1 (after the _ctrl strobe) arms that BRAM:
            # its next read takes a new capture, shared by every BRAM armed with it
            if rising:
                self._armed.add(SNAP_STROBES[name])
                self._snaps.pop(SNAP_STROBES[name], None)
        elif name in ('startAccumulator', 'startSnap', 'startDAC', 'avgIQ_ctrl', 'snapPhase_ctrl',
                      'snapqdr_ctrl', 'ch_we', 'conv_phase_ch_we_Phase', 'conv_phase_snapIQ_ctrl',
                      'conv_phase_snapPhase_ctrl', 'conv_phase_snapI_ctrl', 'conv_phase_snapQ_ctrl'):
            pass  # control strobes: state is read back through self.regs
        return None

    def read_int(self, name):
        if name == 'DRAM_LUT_rd_valid':
            return 0                      # the device LUT is valid as soon as it is written
        if name == 'pulses_addr':
            self._advance_pulses()
            return self.ring.addr
        if name not in self.regs:
            raise RuntimeError('Request read_int failed: no register named %s' % name)
        return self.regs[name]

    def write(self, name, data, offset=0):
        data = bytes(data)
        if name == 'dram_memory':
            I_dac, Q_dac, I_dds, Q_dds = codecs.unpack_luts(data)
            self.cfg.dac_i, self.cfg.dac_q = I_dac, Q_dac
            self.cfg.lut_i, self.cfg.lut_q = lut.deinterleave_dds(I_dds, Q_dds, self.C,
                                                                  self.cfg.dds_lag)
            self.cfg.dirty.add('dds')
            self._t = 0
            self._adc_cache = None
            return None
        m = FIR_RE.match(name)
        if m:
            if len(data) != 4:
                raise RuntimeError('FIR register %s takes 4 bytes' % name)
            self.regs[name] = data
            return None
        self.regs[name] = data
        return None

    def read(self, name, size, offset=0):
        if name == 'avgIQ_bram':
            return self._read_avgiq(size)
        if name == 'snapPhase_bram':
            return self._read_snap_phase(size)
        if name == 'qdr0_memory':
            # longsnapshot: 2 Fix16_13 samples per 32-bit word, '>h' in time order
            raw = self._raw_of(self.regs.get('ch_we', 0), size // 2)
            return raw.astype('>i2').tobytes()[:size]
        if name in SNAP_ROW_BYTES:
            return self._read_conv_phase_snap(name, size)
        if name in ('pulses_bram0', 'pulses_bram1'):
            return self.ring.read(name, size, offset)
        if name in self.regs and isinstance(self.regs[name], bytes):
            return self.regs[name][offset:offset + size]
        raise RuntimeError('Request read failed: no readable register named %s' % name)

    # ---- device side -------------------------------------------------------------------------
    def channelizer(self):
        if self._chan is None:
            if not self.gpu:
                raise RuntimeError('FpgaClient(gpu=False) has no data path')
            from .channelizer import Channelizer
            self._chan = Channelizer(self.C, device=self.device, sample_rate=self.fs,
                                     max_chunk=max(2 * self.N, 1 << 20))
        return self._chan

    def sync(self):
        """Push dirty configuration groups to the device (one ABI call per group)."""
        ch = self.channelizer()
        d = self.cfg
        if 'bins' in d.dirty:
            ch.set_bins(d.bins)
        if 'dds' in d.dirty:
            ch.set_dds(d.lut_i, d.lut_q)
        if 'fir' in d.dirty:
            ch.set_fir(d.fir)
        if 'thr' in d.dirty:
            ch.set_thresholds(np.clip(d.thr, -(1 << 31), (1 << 31) - 1))
        if 'centers' in d.dirty:
            ch.set_centers(d.ic, d.qc)
        if 'baseline' in d.dirty:
            b = d.baseline
            ch.set_baseline(b['mode'], b['alpha'], b['kf'], b['kq'], b['base_thr'])
        d.dirty.clear()
        return ch

    # ---- loop-back source with resonators ---------------------------------
    def set_lo(self, freq):
        """The LO synthesiser (programLOrev2board's ADF4355 SPI writes, ROACH_Setup.py:307-393,
        are control plane): DAC and ADC share it, so moving it moves every tone across its
        resonator while the baseband comb, and so every channel, stays put."""
        self.lo = float(freq)
        self._adc_cache = None

    def set_resonators(self, resonators, lo_nominal):
        """Put MKID resonators on the feedline: a list of dicts of iqsweep.RESDIFF parameters
        (lib/iqsweep.py:824-858: Q, f0, aleak, ph1, da, ang1, Igain, Qgain, Ioff, Qoff). Each DAC
        comb bin passes the resonator whose f0 is nearest its RF frequency at lo_nominal, with
        the complex transmission RESDIFF gives at its RF frequency for the current LO."""
        self.resonators = [dict(r) for r in resonators]
        self.lo_nominal = float(lo_nominal)
        if self.lo is None:
            self.lo = self.lo_nominal
        self._adc_cache = None

    def _adc_lut(self):
        """One 2^16-sample period of the loop-back ADC stream, complex float64: conj(DAC LUT)
        (ROACH_Setup.py:485-487), each comb bin times its resonator's transmission."""
        if self._adc_cache is None:
            x = self.cfg.dac_i.astype(np.float64) - 1j * self.cfg.dac_q.astype(np.float64)
            if self.resonators:
                X = np.fft.fft(x)
                fbb = np.fft.fftfreq(lut.LUT_LEN, 1.0 / self.fs)
                f0 = np.array([r['f0'] for r in self.resonators])
                which = np.argmin(np.abs((self.lo_nominal + fbb)[:, None] - f0[None, :]), axis=1)
                H = np.empty(lut.LUT_LEN, complex)
                for m, r in enumerate(self.resonators):
                    sel = which == m
                    H[sel] = resdiff(self.lo + fbb[sel], **r)
                x = np.fft.ifft(X * H)
            self._adc_cache = x
        return self._adc_cache

    def adc(self, n):
        """Next n loop-back ADC samples: conj(DAC LUT) through the resonators, tiled (+ optional
        AWGN), int16 [n][2]."""
        idx = (self._t + np.arange(n)) % lut.LUT_LEN
        z = self._adc_lut()[idx]
        x = np.stack([z.real, z.imag], axis=1)
        if self.noise_sigma > 0:
            x += self.rng.normal(0, self.noise_sigma, x.shape)
        self._t += n
        return np.clip(np.trunc(x), -32768, 32767).astype(np.int16)

    def _process(self, ch, n_phase_samples):
        """One device call over the next loop-back samples. Like the firmware, the packet stage
        feeds the pulses ring whenever startBuffer is 1, whatever the call was made for."""
        j0 = self._j
        phase, ev = ch.process(self.adc(n_phase_samples * self.N))
        self._j += n_phase_samples
        if self.packet_log is not None:       # test hook: every call's device packets
            self.packet_log.append((ev, j0, n_phase_samples))
        words = self._wire.push(ev, j0, n_phase_samples)
        if self._buffering and len(words):
            self.ring.write(words)
        return phase, ev

    def run(self, n_phase_samples):
        """Stream enough loop-back ADC data for n phase samples per channel; returns
        (phase [n][C], wide packets)."""
        return self._process(self.sync(), n_phase_samples)

    def _read_avgiq(self, size):
        ch = self.sync()
        ch.set_accumulator(False)
        self._process(ch, 64)                    # settle: filters forget the previous LO / LUTs
        ch.set_accumulator(True)                 # startAccumulator 1 after the avgIQ_ctrl strobe
        self._process(ch, 256)                   # accumulate over 256 phase samples
        mi, mq = ch.avg_iq()
        ch.set_accumulator(False)
        words = np.concatenate([np.rint(mi), np.rint(mq)]).astype('>i4')
        return words.tobytes()[:size]

    def _raw_of(self, ch, nsamp):
        """Fix16_13 phase of channel ch for the next nsamp phase samples (device raw values:
        rint(phase * 8192) of the float32 phase, clamped, exactly as k_front quantises). Long
        captures (qdr0_memory: 2^20 samples) stream in pieces of at most 2^24 ADC samples."""
        piece = max(1, (1 << 24) // self.N)
        out = []
        for r0 in range(0, nsamp, piece):
            phase, _ = self.run(min(piece, nsamp - r0))
            out.append(np.clip(np.rint(phase[:, ch] * np.float32(8192)), -25736, 25736).astype(np.int64))
        return np.concatenate(out) if out else np.zeros(0, np.int64)

    def _capture(self, rows):
        """One snapshot capture of the next `rows` phase rows: the low-pass I/Q of the channel
        conv_phase_ch_we_IQ selects (device IQ tap, int16 ADC-count units) and the Fix16_13 phase
        of the channel conv_phase_ch_we_Phase selects, both from the same process calls, so the
        k-th I/Q pair and the k-th phase sample are the same row of the stream (the firmware's
        snap blocks share one capture trigger, readouttesterIQ.py:43-54)."""
        c = self.sync()
        c.set_iq_tap(self.regs.get('conv_phase_ch_we_IQ', 0))
        ph_ch = self.regs.get('conv_phase_ch_we_Phase', 0)
        step = max(1, int(c.cfg.max_chunk) // self.N)
        iq, raw = [], []
        left = rows
        while left > 0:
            n = min(step, left)
            phase, _ = self._process(c, n)
            iq.append(c.iq_tap())
            raw.append(np.clip(np.rint(phase[:, ph_ch] * np.float32(8192)), -25736, 25736))
            left -= n
        iq = np.concatenate(iq).astype(np.int64) if iq else np.zeros((0, 2), np.int64)
        raw = np.concatenate(raw).astype(np.int64) if raw else np.zeros(0, np.int64)
        return dict(I=iq[:, 0], Q=iq[:, 1], phase=raw)

    def _read_conv_phase_snap(self, name, size):
        """conv_phase_snap{I,Q,IQ,Phase}_bram. A BRAM armed by its startSnap strobe is filled by
        one capture taken at the first read after the strobe, shared by every BRAM armed with it
        and held until the next strobe (ROACH_Pulses_IQ.py:375-394 reads I then Q of one capture).
        A BRAM that was never armed free-runs: every read is a fresh capture of its own."""
        rows = size // SNAP_ROW_BYTES[name]
        if name in self._armed:
            cap = self._capture(rows)
            for b in self._armed:
                self._snaps[b] = cap
            self._armed.clear()
        elif name in self._snaps:
            cap = self._snaps[name]
        else:
            cap = self._capture(rows)
        if len(cap['phase']) < rows:
            raise RuntimeError('Request read failed: %s holds %d samples of this capture, %d asked'
                               % (name, len(cap['phase']), rows))
        if name == 'conv_phase_snapIQ_bram':
            return codecs.encode_iq_snap(cap['I'][:rows], cap['Q'][:rows])[:size]
        key = dict(conv_phase_snapI_bram='I', conv_phase_snapQ_bram='Q',
                   conv_phase_snapPhase_bram='phase')[name]
        return codecs.encode_conv_phase_snap(cap[key][:rows])[:size]

    def _read_snap_phase(self, size):
        nsamp = size // 2
        phase, _ = self.run(nsamp)
        ch = self.regs.get('ch_we', 0)
        raw = np.clip(np.rint(phase[:, ch] * np.float32(8192)), -25736, 25736).astype(np.int64)
        return codecs.encode_snap_phase(raw)[:size]

    def _advance_pulses(self):
        """Time passes between two reads of pulses_addr: stream pulse_rows more phase rows."""
        if self._buffering:
            self.run(self.pulse_rows)


def resdiff(x, Q, f0, aleak=0.0, ph1=0.0, da=0.0, ang1=0.0, Igain=1.0, Qgain=1.0, Ioff=0.0, Qoff=0.0):
    """iqsweep.RESDIFF (lib/iqsweep.py:824-858), vectorised: the resonator IQ loop model at
    frequencies x, returned as complex nI + i nQ (the reference returns [nI, nQ] stacked)."""
    dx = (np.asarray(x, np.float64) - f0) / f0
    j2 = 2.0j * Q * dx
    s21b = da * dx + (j2 / (1.0 + j2) - 0.5) + aleak * ((1.0 - np.cos(dx * ph1)) - 1j * np.sin(dx * ph1))
    Ix1 = s21b.real * Igain
    Qx1 = s21b.imag * Qgain
    nI = Ix1 * np.cos(ang1) + Qx1 * np.sin(ang1) + Ioff
    nQ = -Ix1 * np.sin(ang1) + Qx1 * np.cos(ang1) + Qoff
    return nI + 1j * nQ


def _s32(v):
    v = int(v) & 0xFFFFFFFF
    return v - (1 << 32) if v & 0x80000000 else v


class RoachSetup:
    """ROACH_Setup.py AppForm setup methods (GUI values as attributes)."""

    def __init__(self, roach, dac_freqs, lo_freq, attens=None, sample_rate=512e6,
                 n_channels=256, minimum_attenuation=0.0):
        self.roach = roach
        self.dac_freqs = list(dac_freqs)          # spinBox_DACfreq / textedit_DACfreqs
        self.lo_freq = float(lo_freq)             # spinBox_loFreq
        self.sampleRate = float(sample_rate)      # :82
        self.freqRes = self.sampleRate / lut.LUT_LEN  # :83-84
        self.n_channels = n_channels
        self.attens = np.ones(max(n_channels, len(self.dac_freqs))) if attens is None else np.asarray(attens, float)
        self.minimumAttenuation = minimum_attenuation
        self.iq_centers = np.zeros(n_channels, complex)
        self.dacStatus = 'off'

    def freqCombLUT(self, echo, freq, sampleRate, resolution, amplitude=None, phase=None,
                    random_phase='yes'):
        I, Q, sf = lut.freq_comb_lut(echo, freq, sampleRate, resolution, amplitude, phase,
                                     random_phase)
        if echo == 'yes':
            self.scale_factor = sf
        return I, Q

    def define_DAC_LUT(self):
        self.I_dac, self.Q_dac, self.freqs_dac, self.scale_factor, _ = lut.define_dac_lut(
            self.dac_freqs, self.lo_freq, self.attens[:len(self.dac_freqs)], self.sampleRate)

    def define_DDS_LUT(self, phase=None):
        d = lut.define_dds_lut(self.dac_freqs, self.lo_freq, self.n_channels, self.sampleRate,
                               phase=phase, ch_shift=self.roach.cfg.dds_lag)
        self.I_dds, self.Q_dds = d['I_dds'], d['Q_dds']
        self.select_bins_written(d['bins'])
        return d

    def select_bins(self, readout_freqs):
        bins, resid = lut.select_bins(readout_freqs, 2 * self.n_channels, self.sampleRate)
        self.select_bins_written(bins)
        return list(resid)

    def select_bins_written(self, bins):
        for i, b in enumerate(bins):               # ROACH_Setup.py:545-547
            self.roach.write_int('bins', int(b))
            self.roach.write_int('load_bins', (i << 1) + (1 << 0))
            self.roach.write_int('load_bins', (i << 1) + (0 << 0))

    def write_LUTs(self):
        if self.dacStatus == 'off':
            self.roach.write_int('startDAC', 0)
        self.binaryData = codecs.pack_luts(self.I_dac, self.Q_dac, self.I_dds, self.Q_dds)
        self.roach.write('dram_memory', self.binaryData)   # :570

    def define_LUTs(self):
        self.iq_centers = np.zeros(self.n_channels, complex)
        self.define_DAC_LUT()
        self.define_DDS_LUT()
        self.write_LUTs()

    def toggleDAC(self):
        if self.dacStatus == 'off':
            self.roach.write_int('startDAC', 1)
            while self.roach.read_int('DRAM_LUT_rd_valid') != 0:   # :887-895
                self.roach.write_int('startDAC', 0)
                self.roach.write_int('startDAC', 1)
            self.dacStatus = 'on'
        else:
            self.roach.write_int('startDAC', 0)
            self.dacStatus = 'off'

    def findIQcenters(self, I, Q):
        return complex((np.max(I) + np.min(I)) / 2., (np.max(Q) + np.min(Q)) / 2.)

    def loadIQcenters(self):
        for ch in range(self.n_channels):          # :598-605
            center = codecs.center_register(self.iq_centers[ch].real, self.iq_centers[ch].imag)
            self.roach.write_int('conv_phase_centers', center)
            self.roach.write_int('conv_phase_load_centers', (ch << 1) + (1 << 0))
            self.roach.write_int('conv_phase_load_centers', 0)

    def read_avg_iq(self):
        self.roach.write_int('startAccumulator', 0)
        self.roach.write_int('avgIQ_ctrl', 1)
        self.roach.write_int('avgIQ_ctrl', 0)
        self.roach.write_int('startAccumulator', 1)
        data = self.roach.read('avgIQ_bram', 4 * 2 * self.n_channels)
        v = np.frombuffer(data, '>i4').astype(np.float64)
        return v[:self.n_channels], v[self.n_channels:]

    def rotateLoopsReady(self, sweep=None):
        """ROACH_Setup.py:645-671 for every tone channel: DDS phase = arctan2 of the on-resonance
        average IQ (centre-subtracted), then redefine + rewrite the LUTs; sweep = (loSpan, steps)
        re-sweeps the loops afterwards as the reference does (sweepLO, :671)."""
        I, Q = self.read_avg_iq()
        phase = [0.] * self.n_channels
        for n in range(len(self.dac_freqs)):
            phase[n] = np.arctan2(Q[n] - self.iq_centers[n].imag, I[n] - self.iq_centers[n].real)
        self.define_DDS_LUT(phase)
        self.write_LUTs()
        if sweep is not None:        # :670-671 re-sweeps, so the centres follow the rotation
            self.sweepLOready(*sweep)
        return phase

    def programLOrev2board(self, freq=3.2e9, sweep_freq=0, enable=1):
        """ROACH_Setup.py:307-393: the LO at freq (sweep_freq) or at the LO spin box value; the
        ADF4355 register words themselves are control plane (FpgaClient.set_lo)."""
        self.roach.set_lo(freq if sweep_freq else self.lo_freq)

    def sweepLOready(self, loSpan, steps):
        """ROACH_Setup.py:699-810 at one attenuation: step the LO over loSpan in `steps` steps
        (lo_freqs :724), read avgIQ at each step (:767-782), return to the LO (:783), read the
        on-resonance avgIQ and set each tone's IQ centre to the middle of its swept loop
        (findIQcenters, :786-796), and the IQ velocities (:805-810). Returns (I, Q) [N_freqs][steps]."""
        self.N_freqs = len(self.dac_freqs)
        f_base = self.lo_freq
        df = loSpan / steps
        lo_freqs = [f_base + i * df - 0.5 * steps * df for i in range(steps)]
        self.f_span = [[f - 0.5 * steps * df + n * df for n in range(steps)] for f in self.dac_freqs]
        I = np.zeros((self.N_freqs, steps))
        Q = np.zeros((self.N_freqs, steps))
        for i in range(steps):
            self.programLOrev2board(lo_freqs[i], 1)
            Ia, Qa = self.read_avg_iq()
            I[:, i] = Ia[:self.N_freqs]
            Q[:, i] = Qa[:self.N_freqs]
        self.programLOrev2board(f_base, 1)
        Ia, Qa = self.read_avg_iq()
        self.I_on_res, self.Q_on_res = list(Ia[:self.N_freqs]), list(Qa[:self.N_freqs])
        for j in range(self.N_freqs):
            self.iq_centers[j] = self.findIQcenters(I[j], Q[j])
        self.IQ_vels = np.hypot(np.diff(I, axis=1), np.diff(Q, axis=1))
        self.I, self.Q = I, Q
        return I, Q


class RoachPulses:
    """ROACH_Pulses.py AppForm trigger-setup and readback methods."""

    def __init__(self, roach, n_freqs, fir=None, n_channels=256):
        self.roach = roach
        self.N_freqs = n_freqs
        self.n_channels = n_channels
        self.fir = fir                               # importFIRcoeffs result (float taps)
        self.zeroChannels = [0] * n_channels
        self.thresholds = np.zeros(n_channels)
        self.medians = np.zeros(n_channels)
        self.customThresholds = np.full(n_channels, 360.)
        self.scale_to_angle = codecs.SCALE_TO_ANGLE

    def loadFIRcoeffs(self):
        """ROACH_Pulses.py:59-111 (register writes of the 12-bit taps, deleted channels zero)."""
        for ch in range(self.n_channels):
            if ch < self.N_freqs and not self.zeroChannels[ch]:
                taps = codecs.fir_quantise(self.fir)
            else:
                taps = np.zeros(26, np.int64)
            for n, word in enumerate(codecs.fir_registers(taps)):
                self.roach.write('FIR_b%db%d' % (2 * n, 2 * n + 1), word)
                self.roach.write_int('FIR_load_coeff', (ch << 1) + (1 << 0))
                self.roach.write_int('FIR_load_coeff', (ch << 1) + (0 << 0))

    def snapshot_raw(self, ch, steps=10, L=2 ** 10):
        data = b''
        for _ in range(steps):                     # ROACH_Pulses.py:241-248
            self.roach.write_int('ch_we', ch)
            self.roach.write_int('startSnap', 0)
            self.roach.write_int('snapPhase_ctrl', 1)
            self.roach.write_int('snapPhase_ctrl', 0)
            self.roach.write_int('startSnap', 1)
            data += self.roach.read('snapPhase_bram', 4 * L)
        return codecs.decode_snap_phase(data)

    def snapshot_iq(self, ch_we=27, steps=1, L=2 ** 15):
        """ROACH_Pulses_IQ.py:357-407 (snapshot): per step arm conv_phase_snapI/Q, read 4L bytes
        of each BRAM, one '>h' sample per word at bytes [2:4]; phase = arctan2(Q, I) in degrees.
        Returns (Iraw, Qraw, phase)."""
        self.roach.write_int('conv_phase_ch_we_IQ', ch_we)
        bin_i, bin_q = b'', b''
        for _ in range(steps):
            for name, v in (('conv_phase_startSnapI', 0), ('conv_phase_startSnapQ', 0),
                            ('conv_phase_snapI_ctrl', 1), ('conv_phase_snapQ_ctrl', 1),
                            ('conv_phase_snapI_ctrl', 0), ('conv_phase_snapQ_ctrl', 0),
                            ('conv_phase_startSnapI', 1), ('conv_phase_startSnapQ', 1)):
                self.roach.write_int(name, v)
            bin_i += self.roach.read('conv_phase_snapI_bram', 4 * L)
            bin_q += self.roach.read('conv_phase_snapQ_bram', 4 * L)
        Iraw = codecs.decode_conv_phase_snap(bin_i)
        Qraw = codecs.decode_conv_phase_snap(bin_q)
        return Iraw, Qraw, 360 * np.arctan2(Qraw, Iraw) / (2 * np.pi)

    def loadSingleThreshold(self, ch, nsigma=2.5):
        phase = self.snapshot_raw(ch)
        threshold, med = codecs.threshold_from_phase(phase, nsigma)
        self.thresholds[ch] = self.scale_to_angle * threshold
        self.medians[ch] = self.scale_to_angle * med
        if self.customThresholds[ch] != 360.0:
            threshold = max(int(self.customThresholds[ch] / self.scale_to_angle), -25736)
        self.roach.write_int('capture_threshold', threshold)
        self.roach.write_int('capture_load_thresh', (ch << 1) + (1 << 0))
        self.roach.write_int('capture_load_thresh', (ch << 1) + (0 << 0))
        return threshold

    def loadThresholds(self):
        return [self.loadSingleThreshold(ch) for ch in range(self.N_freqs)]

    def _snap_qdr(self, ch, steps, L=2 ** 10, n_qdr=2 ** 19):
        """The snapshot loop shared by longsnapshot and contsnapshot (ROACH_Pulses.py:449-463,
        585-597): per step arm snapPhase + snapqdr, read 2^10 snapPhase words and 2^19 qdr0 words."""
        self.roach.write_int('ch_we', ch)
        snap, qdr = b'', b''
        for _ in range(steps):
            for name, v in (('snapPhase_ctrl', 0), ('snapqdr_ctrl', 0), ('startSnap', 0),
                            ('snapqdr_ctrl', 1), ('snapPhase_ctrl', 1), ('startSnap', 1)):
                self.roach.write_int(name, v)
            snap += self.roach.read('snapPhase_bram', 4 * L)
            qdr += self.roach.read('qdr0_memory', n_qdr * 4)
        for name in ('snapPhase_ctrl', 'snapqdr_ctrl', 'startSnap'):
            self.roach.write_int(name, 0)
        return codecs.decode_snap_phase(snap), codecs.decode_qdr(qdr)

    def longsnapshot(self, ch, steps=1, save_dir=None, n_averages=100, norm1=50.0):
        """ROACH_Pulses.py:433-551: `steps` snapPhase + qdr0 snapshots of channel ch in degrees,
        their statistics, and the qdr stream's phase-noise spectrum over n_averages FFTs
        (521-543; steps=1: 2^20 samples, 10485-point FFTs, the bins of the reference's saved
        ch_noifreqs_0.txt). With save_dir, the reference's text files are written there
        (ch_out_<ch>.txt, ch_snap_<ch>.txt, ch_noifreqs_<ch>.txt, ch_noise_<ch>.txt)."""
        snap_raw, qdr_raw = self._snap_qdr(ch, steps)
        phase = snap_raw * self.scale_to_angle
        qdr_phase = qdr_raw * self.scale_to_angle
        freqs, noise = codecs.noise_spectrum(qdr_phase, n_averages, norm1)
        out = dict(phase=phase, qdr_phase=qdr_phase, noiseFFTFreqs=freqs, noiseFFT=noise,
                   median=float(np.median(phase)), mean=float(np.mean(phase)), std=float(np.std(phase)))
        if save_dir is not None:
            import os
            from datetime import datetime
            os.makedirs(save_dir, exist_ok=True)
            # the reference writes str(q) per line (Python 2: 12 significant digits, codecs.py2_str)
            for name, arr in (('ch_out', qdr_phase), ('ch_snap', phase), ('ch_noifreqs', freqs),
                              ('ch_noise', noise)):
                with open(os.path.join(save_dir, '%s_%d.txt' % (name, ch)), 'w') as f:
                    f.writelines(codecs.py2_str(q) + '\n' for q in arr)
            # and the qdr phase once more under LongSnapShots/ with numpy.savetxt fmt='%.8f'
            # (ROACH_Pulses.py:489-498)
            ls_dir = os.path.join(save_dir, 'LongSnapShots')
            os.makedirs(ls_dir, exist_ok=True)
            out['longsnapshot_file'] = os.path.join(
                ls_dir, 'longsnapshot_' + datetime.utcnow().strftime('%Y-%m-%d_%H%M%S%f')[:-3] + '.txt')
            np.savetxt(out['longsnapshot_file'], qdr_phase, fmt='%.8f')
        return out

    def contsnapshot(self, ch, steps=1, phase_threshold=-20.0, averagelength_power=10, maxloops=None,
                     cap=None):
        """ROACH_Pulses.py:557-762: qdr0 snapshot(s) of channel ch in degrees, then the block-mean
        trigger over it (means of 2^averagelength_power-sample blocks, start 500, hit when
        |mean - x| > phase_threshold, skip 1000, stop at bob + 1500 > len: 614-727) — run on the
        device (mkid_replay_trigger) — and the 2000-sample window [bob-500, bob+1500) of every hit.
        The reference's loop also stops after `maxloops` passes (failsafe, 747-750; its first pass
        always runs, so maxloops <= 1 means one pass); None = no cap. `cap` bounds the device hit list
        (default: every hit the capture can hold, one per 1000 samples).
        Returns dict(pulsenumber, phase (the two columns it saves, '%i %.2f'), hits, total_pulses,
        qdr_phase (the snapshot in degrees))."""
        import torch
        _, qdr_raw = self._snap_qdr(ch, steps)
        qdr_phase = qdr_raw * self.scale_to_angle
        c = self.roach.channelizer()
        dev = c.torch_device()
        d_raw = torch.from_numpy(qdr_raw.astype(np.int16)).to(dev)
        torch.cuda.synchronize(dev)
        if cap is None:
            # the device walks the whole capture (the failsafe is applied to its hit list below),
            # and a hit skips 1000 samples: at most len/1000 + 2 hits
            cap = len(qdr_raw) // 1000 + 2
        hits = replay.block_mean_trigger(c, d_raw, len(qdr_raw), 1, 1, averagelength=2 ** int(averagelength_power),
                                         threshold=float(phase_threshold), start=500, need=1500, skip=1000,
                                         wrap_negative=False, cap=cap)[0]
        if maxloops is not None:
            # pass index of the k-th hit (0-based): every pass advances bob by 1, a hit by 1000;
            # the failsafe breaks after pass failsafe > maxloops - 1, so pass 0 always runs
            passes = max(int(maxloops), 1)
            hits = [h for k, h in enumerate(hits) if (h - 500) - 999 * k < passes]
        pulsenumber = [0.0] * 2000                  # pulse 0's numbers: the initial zeros (560-561)
        final = []
        for k, h in enumerate(hits):
            final.extend(qdr_phase[h - 500:h + 1500].tolist())
            if k > 0:
                pulsenumber.extend([float(k)] * 2000)
        return dict(pulsenumber=pulsenumber, phase=final, hits=hits, total_pulses=len(hits), qdr_phase=qdr_phase)

    def readPulses(self, steps=1):
        """ROACH_Pulses.py:782-832: poll pulses_addr, decode the BRAM ring."""
        self.roach.write_int('startBuffer', 1)
        out = {}
        for _ in range(steps):
            addr0 = self.roach.read_int('pulses_addr')
            addr1 = self.roach.read_int('pulses_addr')
            b0 = self.roach.read('pulses_bram0', 4 * PULSE_RING)
            b1 = self.roach.read('pulses_bram1', 4 * PULSE_RING)
            rng = range(addr0, addr1) if addr1 >= addr0 else \
                list(range(addr0, PULSE_RING)) + list(range(0, addr1))
            for n in rng:
                w1 = struct.unpack('>L', b1[4 * n:4 * n + 4])[0]
                w0 = struct.unpack('>L', b0[4 * n:4 * n + 4])[0]
                out.setdefault(w1 >> 24, []).append(dict(ts=w0 % 2 ** 20, base=(w0 >> 20) % 2 ** 12,
                                                         peak=(w1 >> 12) % 2 ** 12,
                                                         p1=w1 % 2 ** 12 - 2 ** 11))
        self.roach.write_int('startBuffer', 0)
        return out
