import sys, time, torch
sys.path.insert(0, "/root/repo")
from biped_pympc_amd.sharding import ShardedMPC
from biped_pympc_amd.utils.synthetic import make_workload
N, K, B = 10, 10, 4096
wl = make_workload(B, N, seed=1000)
inputs = [torch.from_numpy(x).cuda() for x in wl.inputs]
sh = ShardedMPC(N, K, B, device="cuda", y0=1.0)
for _ in range(5): sh.step(inputs)
torch.cuda.synchronize()
for steps in (10, 20, 50):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    h = []
    for i in range(steps):
        ev[i].record()
        th = time.perf_counter(); sh.step(inputs); h.append(time.perf_counter() - th)
    ev[steps].record()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    per = [ev[i].elapsed_time(ev[i + 1]) for i in range(steps)]
    print(steps, f"wall/step {1e3*el/steps:.4f} ms", "event per step first 3:", [round(x, 4) for x in per[:3]], "median", round(sorted(per)[steps // 2], 4), "host per step us", [round(1e6 * x) for x in h[:3]], round(1e6 * sorted(h)[steps // 2]))
