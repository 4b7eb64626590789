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


class _PersistentSolve:
    """The oracle solve writing into ONE preallocated buffer, as the HIP path's MPCSolveBuffers do:
    a result handed out by reference would be overwritten by the next step."""

    def __init__(self):
        self.buf = None

    def __call__(self, local_inputs):
        x = _oracle_solve(local_inputs)
        if self.buf is None:
            self.buf = torch.empty_like(x)
        self.buf.copy_(x)
        return self.buf


def _rank_main(rank, world, port, total, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        wl = make_workload(total, N, seed=2024, random_gait=True)
        glob = [torch.from_numpy(a) for a in wl.inputs]
        sh = ShardedMPC(N, K, total, device="cpu", solve_fn=_oracle_solve)
        u0 = sh.step(sh.local_slice(glob)).clone()
        u0b = sh.step(sh.local_slice(glob)).clone()  # buffers reused across steps
        # three DIFFERENT steps with their gathers left in flight, results read only at the end and
        # not copied: each handle must own its u0 (send / receive pairs and the solve buffer reused)
        sha = ShardedMPC(N, K, total, device="cpu", solve_fn=_PersistentSolve())
        globs = [[torch.from_numpy(a) for a in make_workload(total, N, seed=3000 + k, random_gait=True).inputs]
                 for k in range(3)]
        hs = [sha.step_async(sha.local_slice(g)) for g in globs]
        u0c = [h.wait() for h in hs]
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
    refs = [_oracle_solve([torch.from_numpy(a) for a in make_workload(total, N, seed=sd, random_gait=True).inputs]
                          ).numpy()[:, 12 * N:12 * N + 12] for sd in (2024, 2024, 3000, 3001, 3002)]
    assert got.shape == (5, total, 12)
    for k in range(5):
        assert np.array_equal(got[k], refs[k]), k


def test_step_async_single_process_results_are_owned():
    """world 1: step_async's handle must not alias the solve buffer the next step overwrites."""
    sh = ShardedMPC(N, K, 4, device="cpu", solve_fn=_PersistentSolve())
    globs = [[torch.from_numpy(a) for a in make_workload(4, N, seed=50 + k).inputs] for k in range(3)]
    hs = [sh.step_async(g) for g in globs]
    for g, h in zip(globs, hs):
        assert torch.equal(h.wait(), _oracle_solve(g)[:, 12 * N:12 * N + 12])


def test_single_process_path_without_process_group():
    wl = make_workload(5, N, seed=9)
    glob = [torch.from_numpy(a) for a in wl.inputs]
    sh = ShardedMPC(N, K, 5, device="cpu", solve_fn=_oracle_solve)
    assert (sh.world, sh.lo, sh.hi) == (1, 0, 5)
    u0 = sh.step(sh.local_slice(glob))
    ref = _oracle_solve(glob)[:, 12 * N:12 * N + 12]
    assert torch.equal(u0, ref)
