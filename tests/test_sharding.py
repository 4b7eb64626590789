"""Multi-process data parallelism on CPU: world_size 2 over gloo.

Each rank solves its shard of one global synthetic batch and the u0 of every env is gathered; the
gathered result must equal a single-process solve of the whole batch bit for bit. The per-rank
solve here is the CPU oracle (tests may call it) standing in for the HIP kernel, so the test
exercises exactly the product sharding / gather code (biped_pympc_amd/sharding.py) that bench.py
and the GPU path use; on MI355X the same class runs over RCCL.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from biped_pympc_amd.sharding import ShardedMPC, shard_bounds
from biped_pympc_amd.utils.synthetic import make_workload

N, K = 10, 5


@pytest.mark.parametrize("total,world", [(0, 1), (1, 2), (7, 3), (4096, 8), (37, 2), (36, 2), (5, 8)])
def test_shard_bounds_partition(total, world):
    spans = [shard_bounds(total, world, r) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == total
    for (l0, h0), (l1, h1) in zip(spans, spans[1:]):
        assert h0 == l1
    sizes = [h - l for l, h in spans]
    assert max(sizes) - min(sizes) <= 1 and min(sizes) >= 0


def test_shard_bounds_rejects_bad_args():
    with pytest.raises(ValueError):
        shard_bounds(10, 0, 0)
    with pytest.raises(ValueError):
        shard_bounds(10, 2, 2)


def _oracle_solve(local_inputs):
    from oracle import oracle
    n = local_inputs[0].shape[0]
    if n == 0:
        return torch.zeros((0, 24 * N), dtype=torch.float64)
    x = oracle.mpc_solve(N, K, [t.numpy() for t in local_inputs], y0=1.0, nthreads=1)[0]
    return torch.from_numpy(x)


def _rank_main(rank, world, port, total, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        wl = make_workload(total, N, seed=2024, random_gait=True)
        glob = [torch.from_numpy(a) for a in wl.inputs]
        sh = ShardedMPC(N, K, total, device="cpu", solve_fn=_oracle_solve)
        u0 = sh.step(sh.local_slice(glob)).clone()
        u0b = sh.step(sh.local_slice(glob)).clone()  # buffers reused across steps
        hs = [sh.step_async(sh.local_slice(glob)) for _ in range(3)]  # gathers left in flight
        u0c = [h.wait().clone() for h in hs]
        if rank == 0:
            np.save(out_path, np.stack([u0.numpy(), u0b.numpy()] + [u.numpy() for u in u0c]))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("total", [37, 36, 1])
def test_gloo_world2_gather_equals_single_process(tmp_path, total):
    out = str(tmp_path / "u0.npy")
    mp.spawn(_rank_main, args=(2, _free_port(), total, out), nprocs=2, join=True)
    got = np.load(out)
    wl = make_workload(total, N, seed=2024, random_gait=True)
    ref = _oracle_solve([torch.from_numpy(a) for a in wl.inputs]).numpy()[:, 12 * N:12 * N + 12]
    assert got.shape == (5, total, 12)
    for k in range(5):
        assert np.array_equal(got[k], ref), k


def test_single_process_path_without_process_group():
    wl = make_workload(5, N, seed=9)
    glob = [torch.from_numpy(a) for a in wl.inputs]
    sh = ShardedMPC(N, K, 5, device="cpu", solve_fn=_oracle_solve)
    assert (sh.world, sh.lo, sh.hi) == (1, 0, 5)
    u0 = sh.step(sh.local_slice(glob))
    ref = _oracle_solve(glob)[:, 12 * N:12 * N + 12]
    assert torch.equal(u0, ref)
