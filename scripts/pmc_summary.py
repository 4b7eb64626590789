"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into profiles/<round>/pmc_*.json.

Usage: python scripts/pmc_summary.py FETCH_CSV WRITE_CSV OUT_JSON --horizon 10 --batch 4096 --iters 10

Per-kernel averages over dispatches. Units and gfx950 corrections follow
/opt/skills/guides/MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE are in KiB;
FETCH_SIZE reports half the bytes of a coalesced read on gfx950 (x2 applied); WRITE_SIZE is exact.
bench.py reads ``pdipm_hbm_bytes_per_launch`` from the JSON as the roofline ``traffic``.
"""
import argparse
import csv
import json
from collections import defaultdict


def per_kernel(path, counter):
    acc = defaultdict(list)
    with open(path) as fh:
        for row in csv.DictReader(fh):
            if row["Counter_Name"] == counter:
                acc[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("fetch_csv")
    p.add_argument("write_csv")
    p.add_argument("out")
    p.add_argument("--horizon", type=int, required=True)
    p.add_argument("--batch", type=int, required=True)
    p.add_argument("--iters", type=int, required=True)
    p.add_argument("--kernel", default="mpc_step_reg_kernel", help="substring of the dominant kernel")
    a = p.parse_args()
    fetch, nf = per_kernel(a.fetch_csv, "FETCH_SIZE")
    write, _ = per_kernel(a.write_csv, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        f_raw = fetch.get(k, 0.0) * 1024.0
        w = write.get(k, 0.0) * 1024.0
        kernels[k] = {"dispatches": nf.get(k, 0), "fetch_size_raw_bytes": f_raw,
                      "fetch_bytes_corrected": 2.0 * f_raw, "write_bytes": w,
                      "hbm_bytes": 2.0 * f_raw + w}
    # the dominant kernel (by name substring) that moved the most bytes
    pd = sorted((v["hbm_bytes"], k) for k, v in kernels.items() if a.kernel in k)
    out = {"horizon": a.horizon, "batch": a.batch, "iters": a.iters,
           "kernel": pd[-1][1] if pd else None,
           "pdipm_hbm_bytes_per_launch": pd[-1][0] if pd else None,
           "correction": "FETCH_SIZE KiB x1024 x2 (gfx950 half-count), WRITE_SIZE KiB x1024",
           "kernels": kernels}
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
