"""CPU sanitizer build of the host planning code (SURVEY.md §5 "Race detection /
sanitizers"): mkids_sdr_amd/csrc/mkid_plan.cpp (workspace sizing, per-call trigger plans, slot order,
tap quantisation, packet merge / re-encode: everything mkid_api.hip computes on the host that sizes or
indexes a device buffer) and oracle/trigger.c, built with -fsanitize=address,undefined
(`make -C mkids_sdr_amd/csrc asan`) and fuzzed by tools/plan_fuzz.cpp against the documented
invariants, the kernels' slot-table writes replayed into exactly-sized buffers."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope='module')
def fuzz_bin():
    r = subprocess.run(['make', '-s', '-C', os.path.join(ROOT, 'mkids_sdr_amd', 'csrc'), 'asan'],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    path = os.path.join(ROOT, 'build', 'asan', 'plan_fuzz')
    assert os.path.exists(path)
    return path


@pytest.mark.parametrize('seed', [1, 2, 3])
def test_plan_fuzz_under_asan_ubsan(fuzz_bin, seed):
    env = dict(os.environ, ASAN_OPTIONS='detect_leaks=1:abort_on_error=0', UBSAN_OPTIONS='print_stacktrace=1')
    r = subprocess.run([fuzz_bin, '400', str(seed)], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert 'plan_fuzz ok' in r.stdout
    assert 'runtime error' not in r.stderr and 'ERROR: AddressSanitizer' not in r.stderr
