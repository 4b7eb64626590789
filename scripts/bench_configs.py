"""Per-GPU rates of every BASELINE.json configuration that runs on the hot path, one MI355X.

python scripts/bench_configs.py [OUT_JSON]      (GPU box; default gpurun_out/configs.json)

bench.py measures config 2 (the headline). This runs bench.py once per configuration at the
per-GPU shard size the multi-GPU configs give each rank (weak scaling: 65536 / 8 = 8192 envs for
config 4, 32768 / 8 = 4096 envs with a randomized gait for config 5), plus config 3 (N = 20), and
collects one record per configuration. Config 1 (batch 1, K = 5, PyTorch-CPU reference plumbing)
is the CPU oracle's case and is not a GPU line.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONFIGS = [
    ("config 2: batch 4096, N=10, 10 iters", []),
    ("config 3: batch 4096, N=20, 10 iters", ["--horizon", "20"]),
    ("config 4 shard: 8192 envs/GPU (65536 over 8), N=10, 10 iters", ["--batch-per-gpu", "8192"]),
    ("config 5 shard: 4096 envs/GPU (32768 over 8), N=10, randomized gait", ["--random-gait"]),
]


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "configs.json")
    rows = []
    for name, args in CONFIGS:
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "30", "--warmup", "5", "--no-dropin", "--no-config3", *args]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
        if r.returncode != 0:
            raise SystemExit(f"{name}: bench.py failed\n{r.stdout}\n{r.stderr}")
        d = json.loads(r.stdout.strip().splitlines()[-1])
        row = {"config": name, "solves_per_s": d["value"], "ms_per_step": d["ms_per_step"],
               "kernel_ms": d["kernels_ms"]["mpc_step_fused"], "roofline_frac_fp64": d["roofline"]["frac"],
               "cpu_baseline_solves_per_s": (d.get("cpu_baseline") or {}).get("value"),
               "parity_max_rel_du": (d.get("parity") or {}).get("max_rel_du")}
        rows.append(row)
        print(json.dumps(row), flush=True)
    with open(out, "w") as fh:
        json.dump(rows, fh, indent=1)


if __name__ == "__main__":
    main()
