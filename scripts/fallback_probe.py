"""Throughput of QPs that are not stage-invariant (the in-launch general fallback) vs the general
kernel and vs a stage-invariant batch.

    python scripts/fallback_probe.py [--horizon 10] [--iters 5]     (GPU; prints one JSON line)

Batches (QPs from qp_former, then A perturbed in one stage's block for the flagged QPs):
  invariant_96      96 QPs, none flagged                      (auto path: register kernel)
  mixed_96          96 QPs, 32 flagged                        (auto: fallback inside the launch)
  all_4096_auto     4096 QPs, every one flagged               (auto: 4096 fallback solves)
  all_4096_general  the same batch on the general kernel      (solver_path("general"))
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from biped_pympc_amd import _native, solver  # noqa: E402
from biped_pympc_amd.utils.synthetic import make_workload, solver_init  # noqa: E402


def qp_batch(B, N, flag_every, seed=77):
    wl = make_workload(B, N, seed=seed)
    ins = [torch.from_numpy(a).cuda() for a in wl.inputs]
    H, f, A, b, G, d = solver.qp_former(ins, N)
    torch.cuda.synchronize()
    if flag_every:
        A = A.clone()
        A[::flag_every, 36 * min(N - 1, 4) + 7] *= 1.0 + 1e-3
    x, s, z, y = (torch.from_numpy(a).cuda() for a in solver_init(d.cpu().numpy(), N))
    return [H, G, A, f, d, b], [x, s, z, y]


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--horizon", type=int, default=10)
    p.add_argument("--iters", type=int, default=5)
    a = p.parse_args()
    N, K = a.horizon, a.iters
    out = {"horizon": N, "iters": K}
    for name, B, every, path in (("invariant_96", 96, 0, "auto"), ("mixed_96", 96, 3, "auto"),
                                 ("invariant_4096", 4096, 0, "auto"), ("all_4096_auto", 4096, 1, "auto"),
                                 ("all_4096_general", 4096, 1, "general")):
        qp, it = qp_batch(B, N, every)
        st = torch.zeros(B, dtype=torch.int32, device="cuda")
        with _native.solver_path(path):
            try:
                ms = timed(lambda: solver.pdipm(qp, it, N, K, status=st))
                flagged = int(((st & _native.STATUS_FALLBACK) != 0).sum())
            except _native.NativeLibraryMissing:  # an earlier build (SRBD_LIB) without the status word
                ms = timed(lambda: solver.pdipm(qp, it, N, K))
                flagged = None
        out[name] = {"ms": round(ms, 4), "qps": B, "fallback_qps": flagged}
        print(name, out[name], file=sys.stderr, flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
