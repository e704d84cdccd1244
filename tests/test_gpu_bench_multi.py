"""Config 4's code path executed on the one-GPU box: bench.py launched as 2 ranks by
torch.distributed.run (one feedline per rank, config-3 geometry: 1024 ch, N = 2048), the
per-step photon-list gather to rank 0 pipelined behind the next step (feedlines.PacketGather),
the barrier + max-over-ranks timing, and rank 0's single JSON line. RCCL needs one GPU per rank,
so the lists move over gloo through pinned host buffers here; the nccl branch (RCCL `gather` of
the device buffers on the side stream) runs as a world-size-1 RCCL group (`--force-gather`).
Both launch forms run: torch.distributed.run, and plain `bench.py --gpus 2` as the driver starts
it (bench.py spawns the ranks itself). Nothing re-execs a process that has touched the GPU. The
reference counterpart: many ROACHes, one PacketMaster (PacketMaster.c:245-405, 577-625)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def test_bench_two_ranks_gloo_gather(gpu):
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2',
           '--master-addr', '127.0.0.1', '--master-port', str(_free_port()),
           os.path.join(ROOT, 'bench.py'), '--gpus', '2', '--backend', 'gloo', '--check-gather',
           '--config', '3', '--log2-samples', '26', '--steps', '3', '--warmup', '1',
           '--no-cpu-baseline', '--copy-mib', '256']
    env = dict(os.environ, MASTER_ADDR='127.0.0.1')
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out['n_gpus'] == 2 and out['steps'] == 3
    assert out['config']['channels'] == 1024 and out['config']['samples_per_step_per_gpu'] == 1 << 26
    g = out['gather']
    assert g['backend'] == 'gloo' and g['ranks'] == 2
    assert g['lists_equal_rank_own'] is True
    assert g['feedlines_distinct'] is True
    assert min(g['last_step_counts']) > 1000
    # every step's lists (warm-up included) reached rank 0
    assert g['packets_gathered_total'] >= 4 * min(g['last_step_counts'])
    assert out['value'] > 0


def _run_bench(args, timeout=110):
    env = {k: v for k, v in os.environ.items()
           if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_PORT', 'LOCAL_WORLD_SIZE')}
    env['MASTER_ADDR'] = '127.0.0.1'
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py')] + args, cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_gpus2_self_launch(gpu):
    """The driver's command line: `bench.py --gpus 2`, no wrapper; backend auto (one GPU for two
    ranks -> gloo)."""
    out = _run_bench(['--gpus', '2', '--check-gather', '--config', '3', '--log2-samples', '26',
                      '--steps', '3', '--warmup', '1', '--no-cpu-baseline', '--copy-mib', '256'])
    assert out['n_gpus'] == 2
    g = out['gather']
    assert g['backend'] == 'gloo' and g['ranks'] == 2
    assert g['lists_equal_rank_own'] is True and g['feedlines_distinct'] is True
    assert min(g['last_step_counts']) > 1000


def test_bench_gpus8_rehearsal(gpu):
    """Config 4's protocol at its real rank count, on the one GPU: plain
    `bench.py --gpus 8` (bench.py spawns the 8 ranks), gloo gather of 8 feedlines' packet lists to
    rank 0 (the reference's 8 boards into one PacketMaster, PacketMaster.c:216-220, 589), and every
    rank's parity witness (its own feedline's first 2^24 samples against the oracle, item 3)."""
    out = _run_bench(['--gpus', '8', '--backend', 'gloo', '--check-gather', '--config', '3',
                      '--log2-samples', '24', '--steps', '3', '--warmup', '1', '--no-cpu-baseline',
                      '--copy-mib', '256'], timeout=280)
    assert out['n_gpus'] == 8
    g = out['gather']
    assert g['backend'] == 'gloo' and g['ranks'] == 8
    assert g['lists_equal_rank_own'] is True and g['feedlines_distinct'] is True
    assert len(g['last_step_counts']) == 8 and min(g['last_step_counts']) > 100
    pr = out['parity_ranks']
    assert [p['rank'] for p in pr] == list(range(8))
    assert out['parity_ranks_green'] is True, pr
    assert all(p['samples'] == 1 << 24 and p['packets_equal_on_device_raw'] for p in pr)


def test_bench_rccl_gather_world1(gpu):
    """The RCCL branch executed: init_process_group('nccl', device_id=...), the gloo control group,
    the device-buffer dist.gather on the side stream, the free-event hand-off, barrier + all_reduce
    timing, all in a world-size-1 group."""
    out = _run_bench(['--gpus', '1', '--force-gather', '--backend', 'nccl', '--check-gather',
                      '--config', '3', '--log2-samples', '26', '--steps', '4', '--warmup', '1',
                      '--no-cpu-baseline', '--copy-mib', '256'])
    assert out['n_gpus'] == 1
    g = out['gather']
    assert g['backend'] == 'nccl' and g['ranks'] == 1
    assert g['lists_equal_rank_own'] is True
    assert g['last_step_counts'][0] > 1000
    assert g['packets_gathered_total'] >= 5 * g['last_step_counts'][0] * 0.9
    assert 'RCCL' in out['config']['parallelism']
