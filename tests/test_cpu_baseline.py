"""bench.py's CPU leg (tools/cpu_baseline.py) on a small case, CPU only: the one-core / all-core
timing legs run, the baseline mode reaches the oracle trigger, and the full-size parity witness
comparison (`parity`) is green for outputs equal to the oracle's and red for a perturbed phase or a
dropped packet."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import signals

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _case(tmp_path, mode):
    C, S = 64, 1 << 16
    case = signals.make_case(C, S, seed=5, pulses_per_ch=3.0)
    quiet = signals.make_case(C, S, seed=5, pulses_per_ch=0)
    thr = signals.thresholds_from_quiet(quiet, signals.oracle_chain(quiet).process(quiet.iq)['raw'])
    inp = str(tmp_path / 'in.npy')
    cfgp = str(tmp_path / 'cfg.npz')
    np.save(inp, case.iq)
    np.savez(cfgp, C=C, pfb=case.pfb, bins=case.bins, lut_i=case.lut_i, lut_q=case.lut_q,
             lpf=case.lpf12, fir=case.fir12, thr=thr, mode=np.int64(mode))
    return case, thr, inp, cfgp


def _witness_from_oracle(case, thr, mode, path, perturb=None):
    from oracle import trigger
    r = signals.oracle_chain(case).process(case.iq)
    ev = trigger.Trigger(case.C, case.fir12, thr, mode=mode).run(r['raw'])[0]
    ph = r['phase'].astype(np.float32)
    if perturb == 'phase':
        ph[20, 3] += 1e-4     # a settled row (>= 16): the 1e-5 rad bar
    if perturb == 'startup':
        ph[3, 3] += 0.1       # row 3 (|y| = 0.006 |y|max, below the IQ floor): the absolute IQ bar
    if perturb == 'packet':
        ev = ev[1:]
    np.savez(path, phase=ph, raw=r['raw'], packets=ev)
    return len(ev)


def _run(inp, cfgp, wit, workers=2):
    cmd = [sys.executable, os.path.join(ROOT, 'tools', 'cpu_baseline.py'), '--input', inp, '--cfg', cfgp,
           '--one-core-samples', str(1 << 16), '--all-core-samples', str(1 << 16), '--workers', str(workers)]
    if wit:
        cmd += ['--witness', wit]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize('mode', [1, 2])
def test_cpu_leg_witness_green(tmp_path, mode):
    case, thr, inp, cfgp = _case(tmp_path, mode)
    wit = str(tmp_path / 'wit.npz')
    npk = _witness_from_oracle(case, thr, mode, wit)
    out = _run(inp, cfgp, wit)
    p = out['parity']
    assert p['green'] is True, p
    assert p['phase_max_err_rad'] < 1e-6 and p['raw_flip_rate'] == 0.0
    assert p['iq_floor_rel'] == 0.01 and p['settled_max_err_above_floor'] < 1e-6
    assert p['settled_tone_samples_below_floor_frac'] <= 0.01
    assert 0 <= p['channels_mostly_below_floor'] <= p['channels_below_floor'] <= 64
    assert p['packets_device'] == p['packets_oracle_chain'] == npk > 0
    assert out['one_core']['value'] > 0 and out['all_cores']['cores'] == 2
    # the mode reached the oracle trigger: the one-core leg counted the witness' packets
    assert ('%d packets' % npk) in out['one_core']['sample']


@pytest.mark.parametrize('perturb', ['phase', 'startup', 'packet'])
def test_cpu_leg_witness_red(tmp_path, perturb):
    case, thr, inp, cfgp = _case(tmp_path, 1)
    wit = str(tmp_path / 'wit.npz')
    _witness_from_oracle(case, thr, 1, wit, perturb=perturb)
    p = _run(inp, cfgp, wit, workers=1)['parity']
    assert p['green'] is False
    if perturb == 'packet':
        assert not p['packets_equal_on_device_raw'] and p['channels_diverged_without_flip'] == 1
    elif perturb == 'phase':
        assert p['phase_max_err_rad'] > 5e-5 and p['phase_max_err_settled_rad'] > 5e-5
    else:
        assert p['phase_max_err_all_rows_rad'] > 5e-2 and p['phase_max_err_settled_rad'] < 1e-6
        assert p['phase_max_err_rad'] < 1e-6 and p['samples_below_floor'] > 0
        assert p['iq_err_below_floor_max_rel'] > p['iq_tol_rel'] == 1e-7
