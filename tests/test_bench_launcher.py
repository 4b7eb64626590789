"""bench.py --gpus N starts its own ranks (the driver runs `python bench.py --gpus N`).

Runs the real bench.py launcher on the CPU: worlds 2, 3 and 8 (the driver's largest) over gloo with
the oracle as the per-rank solve (tests/bench_hook.py), checking the one JSON line, n_gpus = ranks
joined, the per-rank spread (`ranks`), and the gathered u0 in global env order bit for bit against
per-shard oracle solves of the same seeds."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from biped_pympc_amd.utils.synthetic import make_workload

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(hook="tests.bench_hook:oracle_solve", **extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(SRBD_BENCH_SOLVE_HOOK=hook, PYTHONPATH=ROOT, OMP_NUM_THREADS="1", **extra)
    return env


def _run(args, env, timeout=240):
    return subprocess.run([sys.executable, BENCH, *args], env=env, cwd=ROOT, capture_output=True, text=True,
                          timeout=timeout)


@pytest.mark.parametrize("world,B", [(2, 5), (3, 2), (8, 2)])
def test_launcher_starts_ranks_and_gathers_u0(tmp_path, world, B):
    from oracle import oracle
    N, K = 10, 3
    dump = str(tmp_path / "u0.npy")
    r = _run(["--gpus", str(world), "--steps", "2", "--warmup", "1", "--batch-per-gpu", str(B),
              "--iters", str(K), "--dump-u0", dump], _env(), timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == world and line["config"]["global_batch"] == world * B
    assert line["steps"] == 2 and line["value"] > 0
    ranks = line["ranks"]
    assert ranks["joined"] == world
    assert len(ranks["solve_ms_per_rank"]) == world and len(ranks["gather_ms_per_rank"]) == world
    assert 0 < ranks["solve_ms_min"] <= ranks["solve_ms_max"] == max(ranks["solve_ms_per_rank"])
    assert ranks["gather_ms_max"] == max(ranks["gather_ms_per_rank"]) >= 0
    assert ranks["timed_ms_min"] <= ranks["timed_ms_max"]
    assert ranks["timed_ms_max"] == pytest.approx(line["ms_per_step"] * line["steps"], rel=1e-3, abs=1e-3)
    got = np.load(dump)
    ref = np.concatenate([oracle.mpc_solve(N, K, make_workload(B, N, seed=1000 + r_).inputs, y0=1.0, nthreads=1)[0]
                          for r_ in range(world)])[:, 12 * N:12 * N + 12]
    assert got.shape == (world * B, 12)
    assert np.array_equal(got, ref)


def test_gpus_must_match_external_world_size():
    env = _env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0", "--batch-per-gpu", "2"], env)
    assert r.returncode == 2
    assert "WORLD_SIZE=1" in r.stderr


def test_gpus_defaults_to_external_world_size(tmp_path):
    """torchrun --nproc-per-node N bench.py with no --gpus: the launcher's WORLD_SIZE decides (a
    one-rank group here; the external launcher itself is torch.distributed.run)."""
    env = _env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    r = _run(["--steps", "1", "--warmup", "0", "--batch-per-gpu", "2", "--iters", "2"], env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 1 and line["ranks"]["joined"] == 1


def _port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_failing_rank_stops_the_job():
    r = _run(["--gpus", "2", "--steps", "2", "--warmup", "1", "--batch-per-gpu", "2", "--iters", "2"],
             _env(hook="tests.bench_hook:failing_rank1"), timeout=120)
    assert r.returncode != 0
    assert "planted failure on rank 1" in r.stderr
    assert not r.stdout.strip()
