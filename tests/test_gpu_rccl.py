"""RCCL on the MI355X: the product gather path (biped_pympc_amd/sharding.py) under a "nccl" (RCCL)
process group. The GPU box has one device and RCCL refuses two ranks on one device, so this runs a
world-size-1 group: the same all_gather_into_tensor calls (synchronous step and double-buffered
step_async) an 8-GPU job issues, checked bit for bit against the plain fused solve. World size >= 2
is covered over gloo on the CPU (tests/test_sharding.py, tests/test_bench_launcher.py)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CHILD = r"""
import sys, torch, torch.distributed as dist
sys.path.insert(0, sys.argv[1])
from biped_pympc_amd import solver
from biped_pympc_amd.sharding import ShardedMPC
from biped_pympc_amd.utils.synthetic import make_workload
N, K, B = 10, 10, 300
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
assert dist.get_backend() == "nccl"
wls = [[torch.from_numpy(a).cuda() for a in make_workload(B, N, seed=60 + k).inputs] for k in range(3)]
sh = ShardedMPC(N, K, B, device="cuda")
assert sh.collective and sh.world == 1
u0 = sh.step(wls[0]).clone()
hs = [sh.step_async(w) for w in wls]
got = [h.wait() for h in hs]
torch.cuda.synchronize()
for k, w in enumerate(wls):
    ref = solver.mpc_solve(w, N, K, 1.0)[0][:, 12 * N:12 * N + 12]
    assert torch.equal(got[k], ref), k
    if k == 0:
        assert torch.equal(u0, ref)
dist.destroy_process_group()
print("rccl ok")
"""


def test_rccl_world1_gather_path():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29533", RANK="0", WORLD_SIZE="1")
    r = subprocess.run([sys.executable, "-c", _CHILD, ROOT], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "rccl ok" in r.stdout
