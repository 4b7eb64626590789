"""One table over scripts/parity_floor.py reports: per campaign and policy, the failing cases under the
three-restatement floor (and round 5's dense-LU-only floor), the worst ratio to the floor, the envs over
1e-4 in x or u0 beyond 4x their floor, and the recorded / unchecked above-tolerance envs.

    python scripts/floor_summary.py REPORT.floor.json ...
"""
import json
import sys


def main():
    for path in sys.argv[1:]:
        r = json.load(open(path))
        seq = "_ccs sequence" if r["ccs"] else "default sequence"
        print(f"{r['campaign']}: {r['cases']} cases, {r['envs']} envs, {seq}, build {r['build_id']}")
        print(f"  {'policy':18s} {'failing':>7s} {'(dense-only floor)':>18s} {'worst x floor':>13s} "
              f"{'>1e-4 beyond 4x':>15s} {'recorded':>8s} {'unchecked':>9s}")
        for p, v in r["policies"].items():
            print(f"  {p:18s} {v['failed_cases']:7d} {v['failed_cases_dense_floor_only']:18d} "
                  f"{v['worst_ratio_to_floor']:13.1f} {v['envs_over_1e-4_in_x_or_u0_beyond_4x_floor']:15d} "
                  f"{v['above_tol_envs_recorded']:8d} {v['above_tol_unchecked_envs']:9d}")
        print()


if __name__ == "__main__":
    main()
