"""Fused-step kernel time (HIP events) under refinement policies, alternating, B = 4096, K = 10, at
N = 10 and N = 20: the two srbd_set_refinement modes and any scripts/parity_fuzz.py POLICIES entry.

    python scripts/refine_mode_timing.py [POLICY ...]   -> one JSON line per (N, policy, round)
    (default: adaptive strict; REFINE_ROUNDS=3, REFINE_HORIZONS=10,20)
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from biped_pympc_amd import solver  # noqa: E402
from biped_pympc_amd.utils.synthetic import make_workload  # noqa: E402


def ms(fn, reps=50, warm=10):
    for _ in range(warm):
        fn()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    os.environ.setdefault("FUZZ_CCS", "0")
    from parity_fuzz import policy_ctx  # the campaign's policy table (no oracle call here)
    policies = sys.argv[1:] or ["adaptive", "strict"]
    for N in [int(v) for v in os.environ.get("REFINE_HORIZONS", "10,20").split(",")]:
        B, K = 4096, 10
        ins = [torch.from_numpy(a).cuda() for a in make_workload(B, N, seed=1000).inputs]
        bufs = solver.MPCSolveBuffers.allocate(N, B, "cuda")
        for r in range(int(os.environ.get("REFINE_ROUNDS", "3"))):
            for pol in policies:
                with policy_ctx(pol):
                    t = ms(lambda: solver.mpc_solve(ins, N, K, 1.0, buffers=bufs))
                print(json.dumps({"N": N, "policy": pol, "round": r, "ms": round(t, 4),
                                  "solves_per_s": round(B / t * 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
