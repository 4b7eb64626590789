"""GPU: controller step, one launch (srbd_mpc_step) vs three launches, interleaved A/B at B robots."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from biped_pympc_amd.utils.synthetic import make_controller
B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
N = int(sys.argv[2]) if len(sys.argv) > 2 else 10
K = int(sys.argv[3]) if len(sys.argv) > 3 else 10
c = make_controller(B, N, seed=5, device="cuda", n_iter=K)
def t(fn, reps=20):
    for _ in range(3): fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps): fn()
    e1.record(); e1.synchronize()
    return e0.elapsed_time(e1) / reps
for r in range(4):
    print(f"B={B} N={N} K={K} one {t(c.run):.4f} three {t(c.run_three_kernel):.4f}", flush=True)
