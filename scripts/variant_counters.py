"""Diagnostic: time and SQ counters of compile-time variants of the solver (GPU box).

python scripts/variant_counters.py NAME=FLAGS[@CSRC_DIR] [...]
  e.g. base= rep_build=-DSRBD_REPEAT_PHASE=4 old=@/path/to/other/csrc

Each variant: hipcc -> /tmp/libsrbd_mpc_<NAME>.so; ms per launch from scripts/kernel_ab.py
(N=10, B=4096, K=10, auto path = register kernel), then one rocprofv3 --pmc pass of the same command
(SQ_INSTS_VALU, SQ_INSTS_LDS, SQ_LDS_BANK_CONFLICT, SQ_WAVE_CYCLES) summarised per wave.
"""
import csv
import glob
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HORIZON = os.environ.get("VC_N", "10")  # horizon of the measured solver kernel
KERNEL = f"pdipm_srbd_reg_kernel<{HORIZON}>"
COUNTERS = ["SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_WAVE_CYCLES"]


def main():
    rows = []
    for spec in sys.argv[1:]:
        name, _, flags = spec.partition("=")
        flags, _, csrc = flags.partition("@")
        csrc = csrc or os.path.join(ROOT, "biped_pympc_amd/csrc")
        lib = f"/tmp/libsrbd_mpc_{name}.so"
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                        *flags.split(), "-I", os.path.join(ROOT, "include"), "-o", lib,
                        os.path.join(csrc, "srbd_mpc.hip")], check=True)
        env = {**os.environ, "SRBD_LIB": lib}
        cmd = [sys.executable, os.path.join(ROOT, "scripts/kernel_ab.py"), HORIZON, "4096", "10", "auto"]
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            raise SystemExit(f"{name}: kernel_ab failed\n{r.stdout}\n{r.stderr}")
        out = r.stdout
        ms = float([l for l in out.splitlines() if "ms/launch" in l][0].split(":")[1].split("ms")[0])
        d = os.path.join(ROOT, "gpurun_out", f"vc_{name}")
        subprocess.run(["rocprofv3", "--pmc", *COUNTERS, "-d", d, "-o", "run", "--output-format", "csv", "--", *cmd],
                       env=env, capture_output=True, text=True, check=True, timeout=300)
        acc = {c: [] for c in COUNTERS}
        waves = 1
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    if KERNEL in row["Kernel_Name"] and row["Counter_Name"] in acc:
                        acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
                        waves = int(row["Grid_Size"]) // 64  # per wave (a 2-wave QP counts twice)
        vals = {c: (sum(v) / len(v) / waves if v else float("nan")) for c, v in acc.items()}
        rows.append((name, flags, ms, vals))
        print(f"{name:12s} {ms:8.4f} ms  " + "  ".join(f"{c[3:]} {vals[c]:9.0f}" for c in COUNTERS)
              + f"   [{flags}]", flush=True)
    base = rows[0]
    print(f"deltas vs {base[0]}:")
    for name, flags, ms, vals in rows[1:]:
        print(f"{name:12s} {ms - base[2]:+8.4f} ms  " +
              "  ".join(f"{c[3:]} {vals[c] - base[3][c]:+9.0f}" for c in COUNTERS))


if __name__ == "__main__":
    main()
