"""Per-wave SQ counter averages of one kernel from rocprofv3 --pmc CSVs (scripts/gpu_sq_counters.sh).

python scripts/sq_summary.py gpurun_out/pmc_sq gpurun_out/pmc_sq2 [--kernel mpc_step_reg_kernel<10>]

Each counter is averaged over the kernel's dispatches and divided by the waves of one dispatch
(Grid_Size / 64 with one wave per workgroup: one QP per wave). SQ_*_CYCLES / SQ_ACTIVE_* / SQ_WAIT_*
count in quad-cycles (4 clocks) on gfx9; SQ_LDS_BANK_CONFLICT counts clocks the LDS pipe stalled.
"""
import argparse
import csv
import glob
import os
from collections import defaultdict


def main():
    p = argparse.ArgumentParser()
    p.add_argument("dirs", nargs="+")
    p.add_argument("--kernel", default="mpc_step_reg_kernel<10>")
    p.add_argument("--json", help="also write the per-wave averages + derived utilisation here")
    p.add_argument("--waves-per-simd", type=int, default=2)
    p.add_argument("--horizon", type=int, default=10)
    p.add_argument("--batch", type=int, default=4096)
    p.add_argument("--iters", type=int, default=10)
    a = p.parse_args()
    acc, grid = defaultdict(list), {}
    for d in a.dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    if a.kernel in row["Kernel_Name"]:
                        acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
                        grid[row["Counter_Name"]] = int(row["Grid_Size"])
    if not acc:
        raise SystemExit(f"no dispatches of {a.kernel}")
    print(f"kernel {a.kernel}: per-wave averages (one QP per wave)")
    per_wave = {}
    for k in sorted(acc):
        waves = grid[k] // 64
        v = sum(acc[k]) / len(acc[k])
        per_wave[k] = v / waves
        print(f"  {k:24s} {v / waves:12.1f}   (dispatches {len(acc[k])}, waves {waves})")
    if a.json:
        import json
        wc = per_wave.get("SQ_WAVE_CYCLES")
        w = a.waves_per_simd
        util = None
        if wc:
            # a SIMD runs w waves at a time: VALU-active share of the SIMD; LDS-active share of the
            # CU's LDS pipe (4 SIMDs x w waves issue into one LDS)
            util = {"valu_busy": round(w * per_wave.get("SQ_ACTIVE_INST_VALU", 0) / wc, 3),
                    "lds_busy": round(4 * w * per_wave.get("SQ_ACTIVE_INST_LDS", 0) / wc, 3),
                    "waves_per_simd": w}
        json.dump({"kernel": a.kernel, "horizon": a.horizon, "batch": a.batch, "iters": a.iters,
                   "per_wave": per_wave, "utilisation": util}, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
