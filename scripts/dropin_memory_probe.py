"""Diagnostic: device memory of the CusADi drop-in at B envs, with the lazily allocated
CusadiFunction.outputs_dense (product) and with every entry read up front -- what the reference's
_setup allocates for its never-written dense outputs (CusadiFunction.py:77-81).

python scripts/dropin_memory_probe.py [B]     (GPU box) -> one JSON line
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from biped_pympc_amd.cusadi.reference_step import ReferenceQPSchedule  # noqa: E402
from biped_pympc_amd.utils.synthetic import make_workload  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
N = 10
wl = make_workload(B, N, seed=5)
inputs = [torch.from_numpy(a).cuda() for a in wl.inputs]
out = {"batch": B, "horizon": N}
for mode in ("lazy", "eager"):
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    base = torch.cuda.memory_allocated()
    torch.cuda.reset_peak_memory_stats()
    sched = ReferenceQPSchedule(N, B)
    if mode == "eager":  # the reference's allocation: every dense output up front
        for cf in (sched.qp_former, sched.qp_solver):
            for t in cf.outputs_dense:
                t.zero_()
    resident = torch.cuda.memory_allocated() - base
    x = sched.run(inputs)
    torch.cuda.synchronize()
    out[mode] = {"resident_mb": round(resident / 2**20, 1),
                 "peak_mb": round((torch.cuda.max_memory_allocated() - base) / 2**20, 1),
                 "x_checksum": float(x.double().sum())}
    del sched, x
out["peak_saved_mb"] = round(out["eager"]["peak_mb"] - out["lazy"]["peak_mb"], 1)
out["same_solution"] = out["eager"]["x_checksum"] == out["lazy"]["x_checksum"]
print(json.dumps(out))
