"""CPU solve hooks for bench.py's launcher tests (SRBD_BENCH_SOLVE_HOOK="tests.bench_hook:<name>").

The oracle stands in for the HIP solve so that bench.py's own rank launcher, process group and u0
gather run on a machine without a GPU; test infrastructure only (the product never loads this)."""
import os

import torch


def oracle_solve(N, K):
    from oracle import oracle

    def solve(local_inputs):
        x = oracle.mpc_solve(N, K, [t.numpy() for t in local_inputs], y0=1.0, nthreads=1)[0]
        return torch.from_numpy(x)
    return solve


def failing_rank1(N, K):
    """Rank 1 fails in its first solve; rank 0 would then wait in the gather forever unless the
    launcher stops it."""
    inner = oracle_solve(N, K)

    def solve(local_inputs):
        if os.environ.get("RANK") == "1":
            raise RuntimeError("planted failure on rank 1")
        return inner(local_inputs)
    return solve
