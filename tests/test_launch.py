"""bench.py's own multi-rank launch, on the CPU: `python bench.py --gpus N`
without an external launcher starts N fresh rank processes (children of the one process the
driver started, no exec), they rendezvous on 127.0.0.1 and rank 0's single JSON line is relayed.
`--launch-probe` stops each rank after a gloo all-gather, before any GPU call. The reference
counterpart is one PacketMaster connecting to every board (PacketMaster.c:216-218, 577-625)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, 'bench.py')


def _env():
    env = {k: v for k, v in os.environ.items()
           if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_PORT', 'LOCAL_WORLD_SIZE')}
    env['MASTER_ADDR'] = '127.0.0.1'
    return env


def test_bench_spawns_n_ranks():
    r = subprocess.Popen([sys.executable, BENCH, '--gpus', '3', '--launch-probe'], cwd=ROOT, env=_env(),
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    out, err = r.communicate(timeout=120)
    assert r.returncode == 0, err[-2000:]
    lines = [ln for ln in out.splitlines() if ln.strip()]
    assert len(lines) == 1, out
    rec = json.loads(lines[0])
    assert rec['n_gpus'] == 3
    ranks = rec['ranks']
    assert [x['rank'] for x in ranks] == [0, 1, 2]
    assert all(x['world'] == 3 and x['env_rank'] == x['rank'] == x['local_rank'] for x in ranks)
    assert len({x['pid'] for x in ranks}) == 3
    # children of the launching process itself, not re-execs of it
    assert {x['ppid'] for x in ranks} == {r.pid}
    assert r.pid not in {x['pid'] for x in ranks}
    assert all(x['master_addr'] == '127.0.0.1' for x in ranks)


def test_one_gpu_does_not_spawn():
    r = subprocess.run([sys.executable, BENCH, '--gpus', '1', '--launch-probe'], cwd=ROOT,
                       env=dict(_env(), MASTER_PORT='29511', WORLD_SIZE='1', RANK='0'),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    assert rec['n_gpus'] == 1 and rec['ranks'][0]['pid'] != os.getpid()


def test_external_launcher_world_must_match_gpus():
    r = subprocess.run([sys.executable, BENCH, '--gpus', '2', '--launch-probe'], cwd=ROOT,
                       env=dict(_env(), WORLD_SIZE='4', RANK='0', LOCAL_RANK='0', MASTER_PORT='29512'),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert 'WORLD_SIZE=4 but --gpus 2' in r.stderr


def test_failed_rank_fails_the_launch():
    # rank 1 dies before the rendezvous; rank 0 would wait in it forever: the launcher must stop
    # rank 0, return rank 1's status and print no JSON line
    r = subprocess.run([sys.executable, BENCH, '--gpus', '2', '--launch-probe'], cwd=ROOT,
                       env=dict(_env(), MKID_PROBE_FAIL_RANK='1'),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 3, r.stderr[-2000:]
    assert 'rank 1 exited with 3' in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith('{')]


def test_backend_auto_resolution(monkeypatch):
    """--backend auto: RCCL when device_count() >= world (one GPU per rank, the
    driver's 8-GPU node), gloo when ranks must share a GPU (the one-GPU rehearsal); an explicit
    backend is kept. device_count() is mocked: no GPU is touched."""
    import torch
    import bench
    monkeypatch.setattr(torch.cuda, 'device_count', lambda: 8)
    assert bench.resolve_backend('auto', 8) == 'nccl'
    assert bench.resolve_backend('auto', 2) == 'nccl'
    assert bench.resolve_backend('gloo', 8) == 'gloo'
    monkeypatch.setattr(torch.cuda, 'device_count', lambda: 1)
    assert bench.resolve_backend('auto', 8) == 'gloo'
    assert bench.resolve_backend('auto', 2) == 'gloo'
    assert bench.resolve_backend('auto', 1) == 'nccl'
    assert bench.resolve_backend('nccl', 8) == 'nccl'
    assert bench.resolve_backend('auto', 4, device_count=4) == 'nccl'
