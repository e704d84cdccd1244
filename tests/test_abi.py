"""The C ABI library loads and exports every symbol include/mkidgpu.h declares (no GPU calls)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, 'include', 'mkidgpu.h')


def declared():
    src = open(HEADER).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return sorted(set(re.findall(r'\b(mkid_[a-z_]+)\s*\(', src)))


def test_header_matches_binding():
    from mkids_sdr_amd import _lib
    assert declared() == _lib.EXPORTS


def test_library_exports_every_declared_symbol():
    from mkids_sdr_amd import _lib
    L = _lib.load()
    for name in declared():
        assert hasattr(L, name), name
    out = subprocess.check_output(['nm', '-D', '--defined-only', _lib.LIB_PATH]).decode()
    exported = set(re.findall(r'\bT (mkid_[a-z_]+)\b', out))
    assert set(declared()) <= exported


def test_host_only_entry_points():
    """Entry points that touch no GPU: default config, packet re-encode, error paths."""
    from mkids_sdr_amd import _lib
    L = _lib.load()
    cfg = _lib.Cfg()
    assert L.mkid_default_cfg(ctypes.byref(cfg), 1024) == 0
    assert (cfg.fft_len, cfg.dds_entries, cfg.pfb_taps, cfg.fir_taps) == (2048, 64, 4, 26)
    assert L.mkid_default_cfg(ctypes.byref(cfg), 100) == _lib.MKID_E_ARG
    assert L.mkid_kernel_name(0) == b'k_channelize'
    import numpy as np
    from mkids_sdr_amd import codecs
    w = np.array([(3 << 52) | (1500 << 40) | (1900 << 28) | 123456], np.uint64)
    out = np.zeros(1, np.uint64)
    assert L.mkid_pack_reference(w.ctypes.data_as(ctypes.c_void_p), 1,
                                 out.ctypes.data_as(ctypes.c_void_p)) == 0
    assert out[0] == codecs.wide_to_reference(w)[0]
    bad = np.array([300 << 52], np.uint64)
    assert L.mkid_pack_reference(bad.ctypes.data_as(ctypes.c_void_p), 1,
                                 out.ctypes.data_as(ctypes.c_void_p)) == _lib.MKID_E_ARG


def test_create_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip('GPU present: covered by the -m gpu suite')
    from mkids_sdr_amd import _lib
    from mkids_sdr_amd.channelizer import Channelizer
    with pytest.raises(_lib.MkidError):
        Channelizer(64)
