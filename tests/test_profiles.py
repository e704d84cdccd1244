"""The roofline evidence chain: bench.py reads `roofline.traffic` and
`avg_launch_ms_rocprof` from profiles/pmc_traffic.json / kernel_avg_ms.json by config. Every entry
must come from a profile run of its own config (tools/prof_meta.py reads the config from the run's
bench line), and the committed per-kernel summary it names must hold the same counter value."""
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_pmc_traffic_entries_match_their_config():
    rec = json.load(open(os.path.join(ROOT, 'profiles', 'pmc_traffic.json')))
    assert 'config3' in rec and 'k_front' in rec['config3']
    for key, kernels in rec.items():
        cfg = int(key[len('config'):])
        for name, e in kernels.items():
            assert e['bench_config'] == cfg, (key, name, e)
            summ = os.path.join(ROOT, e['summary'])
            assert os.path.exists(summ), summ
            lines = {ln.split(' ', 1)[0]: json.loads(ln.split(' ', 1)[1])
                     for ln in open(summ) if ln.strip()}
            assert lines[name]['hbm_bytes_per_launch'] == e['hbm_bytes_per_launch'], (key, name)
            assert abs(e['hbm_bytes_per_sample'] * e['pmc_samples'] - e['hbm_bytes_per_launch']) < 1.0
    # the config-3 and config-5 front ends are different kernels: their counters must differ
    if 'config5' in rec:
        assert rec['config3']['k_front']['hbm_bytes_per_launch'] != rec['config5']['k_front']['hbm_bytes_per_launch']


def test_kernel_avg_entries_match_their_config():
    rec = json.load(open(os.path.join(ROOT, 'profiles', 'kernel_avg_ms.json')))
    for key, e in rec.items():
        assert e['bench_config'] == int(key[len('config'):]), (key, e)
        assert 'k_front' in e and e['k_front'] > 0


def test_prof_meta_files_runs_under_their_own_config(tmp_path):
    import sys
    sys.path.insert(0, os.path.join(ROOT, 'tools'))
    import prof_meta
    d = tmp_path / 'prof_x'
    d.mkdir()
    (d / 'kt.log').write_text('noise\n' + json.dumps({'config': {'config': 5, 'samples_per_step_per_gpu': 1 << 30}}) + '\n')
    assert prof_meta.resolve(str(d)) == (5, 1 << 30)
    assert prof_meta.resolve_config(str(d)) == 5
    import pytest
    with pytest.raises(SystemExit):
        prof_meta.resolve(str(d), 3)
    with pytest.raises(SystemExit):
        prof_meta.resolve(str(tmp_path))
