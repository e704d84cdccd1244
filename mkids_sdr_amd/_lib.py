"""ctypes binding of libmkidgpu.so (include/mkidgpu.h).

The shared library is the product: it is built in-tree (``mkids_sdr_amd/libmkidgpu.so``) by
``__graft_entry__.build()`` / ``make -C mkids_sdr_amd/csrc``. There is no CPU fallback: importing
the binding without the library, or creating a context without a GPU, raises.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# MKID_LIB: a build variant to test in place of the in-tree library (tools/build_variant.sh A/Bs)
LIB_PATH = os.environ.get('MKID_LIB') or os.path.join(HERE, 'libmkidgpu.so')

MKID_OK = 0
MKID_E_ARG = -1
MKID_E_HIP = -2
MKID_E_STATE = -3
MKID_E_OVERFLOW = -4
MKID_E_NODEV = -5

BASE_NONE, BASE_EMA, BASE_SVF = 0, 1, 2
K_CHANNELIZE, K_FIR_PHASE, K_TRIGGER, K_COMPACT, K_FRONT, K_COPY, K_HEIGHTS, K_COUNT = 0, 1, 2, 3, 4, 5, 6, 7
FRONT_AUTO, FRONT_SPLIT = 0, 1

PKT_CH_SHIFT, PKT_PEAK_SHIFT, PKT_BASE_SHIFT = 52, 40, 28
PKT_TS_MASK = (1 << 28) - 1


class MkidError(RuntimeError):
    """Raised on a negative MKID_E_* return code (katcp raises RuntimeError too:
    pulse_triggering_v2.py:177-179 catches it)."""

    def __init__(self, code, msg):
        super().__init__('%s (code %d)' % (msg, code))
        self.code = code


class Cfg(ctypes.Structure):
    _fields_ = [('n_channels', ctypes.c_int32), ('fft_len', ctypes.c_int32),
                ('pfb_taps', ctypes.c_int32), ('fir_taps', ctypes.c_int32),
                ('dds_entries', ctypes.c_int32), ('dead_time', ctypes.c_int32),
                ('max_events_per_ch', ctypes.c_int32), ('front', ctypes.c_int32),
                ('max_chunk', ctypes.c_int64), ('sample_rate', ctypes.c_double)]


REPLAY_ROLLING, REPLAY_BLOCK = 0, 1


class ReplayCfg(ctypes.Structure):
    _fields_ = [('mode', ctypes.c_int32), ('length', ctypes.c_int32), ('start', ctypes.c_int32),
                ('need', ctypes.c_int32), ('skip', ctypes.c_int32), ('wrap_negative', ctypes.c_int32),
                ('threshold_deg', ctypes.c_double)]


class TemplateInfo(ctypes.Structure):
    _fields_ = [('count', ctypes.c_double), ('count1', ctypes.c_double), ('pm', ctypes.c_double),
                ('pdev', ctypes.c_double), ('flag', ctypes.c_int32), ('pstart', ctypes.c_int32)]


class SynthTone(ctypes.Structure):
    _fields_ = [('amp', ctypes.c_float), ('phase0', ctypes.c_float),
                ('freq_index', ctypes.c_int32), ('pad', ctypes.c_int32)]


class Pulse(ctypes.Structure):
    _fields_ = [('start', ctypes.c_int64), ('tone', ctypes.c_int32), ('amp_rad', ctypes.c_float)]


P = ctypes.c_void_p
I32, I64 = ctypes.c_int32, ctypes.c_int64
_SIGS = {
    'mkid_default_cfg': [P, I32],
    'mkid_create': [P, I32, P],
    'mkid_destroy': [P],
    'mkid_get_cfg': [P, P],
    'mkid_set_stream': [P, P],
    'mkid_set_pfb': [P, P, I32],
    'mkid_pfb_effective_taps': [P, I32, I32, P, P],
    'mkid_slot_order': [P, I32, P],
    'mkid_set_bins': [P, P, I32],
    'mkid_set_dds': [P, P, P, I32],
    'mkid_set_lpf': [P, P, I32],
    'mkid_set_fir': [P, P, I32, I32],
    'mkid_set_centers': [P, P, P, I32],
    'mkid_set_thresholds': [P, P, I32],
    'mkid_set_baseline': [P, I32, I32, I32, I32, I32],
    'mkid_set_rearm': [P, I32],
    'mkid_reset_stream': [P],
    'mkid_process': [P, P, I64, P, P, I64, P],
    'mkid_process_device': [P, P, I64, P, P, I64, P],
    'mkid_trigger_phase': [P, P, I64, P, I64, P],
    'mkid_last_raw_phase': [P, P, P],
    'mkid_read_raw_phase': [P, P, I64, P],
    'mkid_set_iq_tap': [P, I32],
    'mkid_read_iq_tap': [P, P, I64, P],
    'mkid_set_accumulator': [P, I32],
    'mkid_avg_iq': [P, P, P],
    'mkid_trigger_reruns': [P, P],
    'mkid_pack_reference': [P, I64, P],
    'mkid_set_timing': [P, I32],
    'mkid_set_timing_mask': [P, ctypes.c_uint32],
    'mkid_get_timing': [P, I32, P, P],
    'mkid_replay_trigger': [P, P, I64, I64, I32, P, P, I32, P],
    'mkid_make_template': [P, P, P, I64, P, P, P],
    'mkid_optimal_filter': [P, P, P, I32, I32, P],
    'mkid_set_pulse_filter': [P, P, I32, I32, I32],
    'mkid_pulse_heights': [P, P, I64, I64, P, I64, P],
    'mkid_pulse_heights_counted': [P, P, I64, I64, P, P, I64, P],
    'mkid_stream_copy': [P, P, P, I64],
    'mkid_synth_adc': [P, P, I64, I64, P, P, P, I64, ctypes.c_float, ctypes.c_float, I32,
                       ctypes.c_float, ctypes.c_uint32],
}
# every symbol include/mkidgpu.h declares (tests/test_abi.py checks the header against this)
EXPORTS = sorted(list(_SIGS) + ['mkid_last_error', 'mkid_global_error', 'mkid_kernel_name'])

_lib = None


def load(path=None):
    """Load the in-tree HIP library; raise if it was not built. `path` loads a build variant
    (tools/kbench.py) as a separate library instance."""
    global _lib
    if path is None and _lib is not None:
        return _lib
    lp = path or LIB_PATH
    if not os.path.exists(lp):
        raise ImportError('libmkidgpu.so not built at %s: run __graft_entry__.build() '
                          '(make -C mkids_sdr_amd/csrc); there is no CPU fallback' % lp)
    L = ctypes.CDLL(lp)
    for name, args in _SIGS.items():
        if path is not None and not hasattr(L, name):
            continue  # an older build variant (tools/kbench.py A/B) may predate a symbol
        f = getattr(L, name)
        f.argtypes = args
        f.restype = ctypes.c_int
    for name in ('mkid_last_error',):
        getattr(L, name).argtypes = [P]
        getattr(L, name).restype = ctypes.c_char_p
    L.mkid_global_error.argtypes = []
    L.mkid_global_error.restype = ctypes.c_char_p
    L.mkid_kernel_name.argtypes = [I32]
    L.mkid_kernel_name.restype = ctypes.c_char_p
    if path is None:
        _lib = L
    return L


def check(rc, ctx=None):
    if rc != MKID_OK:
        L = load()
        msg = (L.mkid_last_error(ctx) if ctx else L.mkid_global_error()) or b''
        raise MkidError(rc, msg.decode(errors='replace'))
    return rc
