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


@pytest.mark.parametrize('C', [1024, 2048])
def test_slot_order_host(C):
    """The select-slot order of k_front3 / k_front5 (mkid_slot_order): a permutation that keeps
    each wave's 128 channels, matches tools/lds_assign.py's model, and cuts the modelled Y-gather
    LDS cycles (one per distinct address on the busiest bank pair of each 32-lane half) by >= 35 %."""
    import numpy as np
    from mkids_sdr_amd import _lib
    from tools.lds_assign import (f5_groups, f5_key, f5_waves, group_cost, natural_groups,
                                  slot_order_blocks, slot_order_f5_waves, yswz)
    L = _lib.load()
    rng = np.random.default_rng(11)
    for trial in range(2):
        bins = rng.permutation(np.arange(1, 2 * C))[:C].astype(np.int32)
        out = np.zeros(C, np.int16)
        assert L.mkid_slot_order(bins.ctypes.data_as(ctypes.c_void_p), C, out.ctypes.data_as(ctypes.c_void_p)) == 0
        o = out.astype(np.int64)
        assert np.array_equal(np.sort(o), np.arange(C))
        slots = np.arange(C)
        if C == 1024:   # k_front3: wave w keeps channels 128 w ..
            assert np.array_equal(o // 128, (slots % (C // 2)) // 64)
            assert np.array_equal(o, slot_order_blocks(bins, C=C))
            yo = np.array([yswz(int(b) & 511) for b in bins])
            nat, opt = group_cost(natural_groups(C), yo), group_cost(natural_groups(C), yo[o])
        else:           # k_front5: each select wave keeps the natural channels of its slots, and
            # every channel is base + l + stride q (the kernel's packed 8-bit (q, l) code)
            for base, stride, nq in f5_waves():
                own = np.array([base + l + stride * q for q in range(nq) for l in range(64)])
                assert np.array_equal(np.sort(o[own]), np.sort(own))
            assert np.array_equal(o, slot_order_f5_waves(bins))
            key = f5_key(bins)
            nat, opt = group_cost(f5_groups(), key), group_cost(f5_groups(), key[o])
        assert opt <= 0.65 * nat, (nat, opt)
    ident = np.zeros(256, np.int16)
    assert L.mkid_slot_order(np.arange(256, dtype=np.int32).ctypes.data_as(ctypes.c_void_p), 256,
                             ident.ctypes.data_as(ctypes.c_void_p)) == 0
    assert np.array_equal(ident, np.arange(256))


def test_create_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip('GPU present: covered by the -m gpu suite')
    from mkids_sdr_amd import _lib
    from mkids_sdr_amd.channelizer import Channelizer
    with pytest.raises(_lib.MkidError):
        Channelizer(64)


def test_front5_select_groups_cover_every_channel_once():
    """k_front5's select-read groups (tools/lds_assign.f5_groups: waves 4-11 with three channels per
    thread, 12-15 with two) hold each of the 2048 channels exactly once, and the relabel order
    used for its conflict bound (slot_order_f5) is a permutation that does not raise the modelled
    gather cost."""
    import numpy as np
    from tools.lds_assign import f5_groups, group_cost, slot_order_f5, yswz
    g = f5_groups()
    assert len(g) == 64 and all(len(x) == 32 for x in g)
    assert sorted(c for x in g for c in x) == list(range(2048))
    rng = np.random.default_rng(3)
    bins = rng.permutation(np.arange(1, 4096))[:2048]
    perm = slot_order_f5(bins)
    assert sorted(perm.tolist()) == list(range(2048))
    yoff = np.array([yswz(int(b) & 511) for b in bins])
    assert group_cost(g, yoff[perm]) <= group_cost(g, yoff)
