"""bench.py --gpus N: the launcher the driver's scaling runs go through.

Without WORLD_SIZE and N > 1, bench.py starts N child ranks under torch.distributed.run and
relays rank 0's line; with WORLD_SIZE set it must equal N; with fewer GPUs than N it refuses.
The self-test mode runs the same launcher with gloo ranks and no GPU."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, 'bench.py')


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_ADDR',
                                                           'MASTER_PORT')}
    env.update(kw)
    return env


def _run(args, env, timeout=240):
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True, text=True, timeout=timeout)


def test_launcher_starts_n_ranks_and_prints_one_line():
    r = _run(['--gpus', '2', '--launch-selftest'], _env())
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out['n_gpus'] == 2 and out['rccl_world'] == 2
    assert out['ranks'] == [0, 1]
    assert out['rank_sum'] == 3.0               # both ranks joined the collective
    assert out['pid'] != os.getpid()


def test_world_size_mismatch_exits_nonzero():
    r = _run(['--gpus', '2', '--launch-selftest'], _env(WORLD_SIZE='1', RANK='0', LOCAL_RANK='0'))
    assert r.returncode != 0
    assert 'WORLD_SIZE=1' in r.stderr
    assert '"n_gpus"' not in r.stdout


def test_too_few_gpus_exits_nonzero():
    """this container has no GPU: a 2-GPU request is refused before any rank starts"""
    r = _run(['--gpus', '2'], _env(HIP_VISIBLE_DEVICES=''))
    assert r.returncode != 0
    assert 'needs 2 GPUs' in r.stderr
    assert '"n_gpus"' not in r.stdout
