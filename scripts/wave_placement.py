"""Diagnostic: where and when each QP's wave ran (HW_ID, XCC_ID, s_memrealtime start / end), from
a -DSRBD_HWID_DUMP build of the fused kernel (the residual output slots carry the values).

python scripts/wave_placement.py [B]      (GPU box; builds /tmp/libsrbd_mpc_hwid.so; WP_FLAGS=extra -D)
"""
import collections
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
lib = "/tmp/libsrbd_mpc_hwid.so"
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                "-DSRBD_HWID_DUMP", *os.environ.get("WP_FLAGS", "").split(), "-I", os.path.join(ROOT, "include"), "-o", lib,
                os.path.join(ROOT, "biped_pympc_amd/csrc/srbd_mpc.hip")], check=True)
os.environ["SRBD_LIB"] = lib
import numpy as np  # noqa: E402
import torch  # noqa: E402

from biped_pympc_amd import solver  # noqa: E402
from biped_pympc_amd.utils.synthetic import make_workload  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
N, K = 10, 10
wl = make_workload(B, N, seed=1)
ins = [torch.from_numpy(a).cuda() for a in wl.inputs]
for _ in range(30):
    out = solver.mpc_solve(ins, N, K)
torch.cuda.synchronize()
r = out[4].cpu().numpy()
hw = r[:, 0].astype(np.int64)
xcc = r[:, 1].astype(np.int64)
t0, t1 = r[:, 2] - r[:, 2].min(), r[:, 3] - r[:, 2].min()  # 100 MHz ticks
wave, simd, cu, sh, se = hw & 15, (hw >> 4) & 3, (hw >> 8) & 15, (hw >> 12) & 1, (hw >> 13) & 7
print(f"B={B}: span {t1.max() / 100:.1f} us; per-wave duration median {np.median(t1 - t0) / 100:.1f} us, "
      f"min {np.min(t1 - t0) / 100:.1f}, max {np.max(t1 - t0) / 100:.1f}")
print("start-time histogram (us):", np.histogram(t0 / 100, bins=10)[0].tolist(),
      "edges", np.round(np.histogram(t0 / 100, bins=10)[1], 1).tolist())
per_simd = collections.defaultdict(list)
for e in range(B):
    per_simd[(xcc[e], se[e], sh[e], cu[e], simd[e])].append((t0[e] / 100, t1[e] / 100, int(wave[e]), e))
print("distinct SIMDs", len(per_simd), "waves per SIMD", collections.Counter(len(v) for v in per_simd.values()))
print("wave-slot ids", collections.Counter(int(w) for w in wave))
for key in list(per_simd)[:6]:
    print(key, sorted((round(a, 1), round(b, 1), w, e) for a, b, w, e in per_simd[key]))
# overlap of the two waves that start together on a SIMD
starts = [sorted(v)[:2] for v in per_simd.values() if len(v) >= 2]
d = np.array([abs(a[0][0] - a[1][0]) for a in starts])
print(f"first two waves per SIMD: start offset median {np.median(d):.2f} us, max {d.max():.2f}")
