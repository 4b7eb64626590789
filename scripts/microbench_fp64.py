"""Run scripts/microbench_fp64.hip on the GPU box and print the measured FP64 facts.

python scripts/microbench_fp64.py   (builds /tmp/libmicrobench_fp64.so with hipcc for gfx950)
"""
import ctypes
import os
import struct
import subprocess

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = "/tmp/libmicrobench_fp64.so"
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-o", LIB,
                os.path.join(HERE, "microbench_fp64.hip")], check=True)
L = ctypes.CDLL(LIB)

torch.cuda.init()
n = 1 << 22
rng = np.random.default_rng(0)
x = np.exp(rng.uniform(np.log(1e-12), np.log(1e12), n)) * rng.choice([-1.0, 1.0], n)
xd = torch.from_numpy(x).cuda()
out = torch.zeros(7, dtype=torch.int64, device="cuda")
assert L.run_acc(ctypes.c_void_p(xd.data_ptr()), ctypes.c_int(n), ctypes.c_void_p(out.data_ptr())) == 0
torch.cuda.synchronize()
o = out.cpu().numpy()
f = [struct.unpack("<d", struct.pack("<q", int(v)))[0] for v in o[:3]]
print(f"v_rcp_f64 accuracy over {n} log-uniform |x| in [1e-12, 1e12]:")
print(f"  max |x r - 1|: raw {f[0]:.3e}, +1 Newton {f[1]:.3e}, +2 Newton {f[2]:.3e} (ulp(1) = 2.2e-16)")
print(f"  r != correctly rounded 1/x: 1 Newton {o[3]} / {n}, 2 Newton {o[4]} / {n}")
f3 = struct.unpack("<d", struct.pack("<q", int(o[5])))[0]
print(f"  cubic step y(1+e+e^2): max |x r - 1| {f3:.3e}, != 1/x: {o[6]} / {n}")
cyc = torch.zeros(10, dtype=torch.int64, device="cuda")
sink = torch.zeros(64, dtype=torch.float64, device="cuda")
for _ in range(2):
    assert L.run_lat(ctypes.c_void_p(cyc.data_ptr()), ctypes.c_void_p(sink.data_ptr())) == 0
torch.cuda.synchronize()
c = cyc.cpu().numpy() / 256.0
print("one wave64, s_memtime cycles per chain link (256 links):")
print(f"  dependent v_fma_f64            {c[0]:6.1f}")
print(f"  v_mov_b64_dpp -> v_fma_f64     {c[1]:6.1f}")
print(f"  dependent v_rcp_f64            {c[2]:6.1f}")
print(f"  ds_bpermute (double) -> fma    {c[3]:6.1f}")
print(f"  independent v_fma_f64 (8 ILP)  {c[4]:6.1f}  (issue cost per instruction)")
print(f"  dependent v_mov_b64_dpp        {c[5]:6.1f}")
print(f"  independent v_mov_b64_dpp      {c[6]:6.1f}  (issue cost per instruction)")
print(f"  LDS store -> broadcast read -> fma {c[7]:6.1f}")
print(f"  v_fmac_f64_dpp (fused, 8 indep.) {c[8]:6.1f}  per instruction incl. 1 s_nop per 8")
print(f"  v_mov_b64_dpp + v_fmac_f64       {c[9]:6.1f}  per pair")
