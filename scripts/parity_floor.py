"""Offline floor check of a parity campaign (scripts/parity_fuzz.py output), on the CPU host.

    python scripts/parity_floor.py CAMPAIGN.json.gz [OUT_JSON]     (default: CAMPAIGN's name + .floor.json)
    FLOOR_WORKERS=8             processes (single-threaded BLAS / oracle each)
    FLOOR_CACHE=path.json.gz    floors already computed (keyed by campaign sequence, seed and env), reused
    FLOOR_MAX_FAILS=200         a policy outside the campaign's full-record set stops being checked after
                                this many failing cases (it is rejected; its other cases count as unverified)

The campaign records every env outside its bounds (x, s, z, y beyond the K tolerance, or u0 beyond 1e-4)
with its five errors against the oracle. Each such env passes only within 4x its own FP64 floor: per
output, the larger distance from the checker (the sparse LDL^T under exact minimum degree) of the two
other CPU restatements -- the same LDL^T under AMD, the ordering of the reference's ca.ldl
(sparse_pdipm_solver.py:451), and dense LU with partial pivoting (oracle/pdipm_dense.py) -- on that env
(DESIGN.md 4). This script computes that floor for EVERY recorded env of the policies the campaign
recorded in full (the two refinement modes by default): a case is ok only when all of its recorded envs
were checked and passed; the summary then carries above_tol_unchecked_envs = 0 for them. For the other
policies a case stops at its first failing env (enough to reject it). Test infrastructure only.
"""
import os

os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")
os.environ.setdefault("OMP_NUM_THREADS", "1")

import gzip  # noqa: E402
import importlib  # noqa: E402
import json  # noqa: E402
import sys  # noqa: E402
import time  # noqa: E402
from multiprocessing import Pool  # noqa: E402

import numpy as np  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))

_PF = None  # scripts/parity_fuzz, imported with the campaign's FUZZ_CCS (its draw sequence depends on it)
_PARAMS = {}


def _init(ccs, params):
    global _PF, _PARAMS
    os.environ["FUZZ_CCS"] = "1" if ccs else "0"
    _PF = importlib.import_module("parity_fuzz")
    _PARAMS = params


def floors_of(task):
    """(seed, [env, ...]) -> {env: [x, s, z, y, u0] floors} (parity_fuzz.floor_env)."""
    seed, envs = task
    N, K, B, entry, path, kw, y0, extra = _PARAMS[seed]
    _, ins = _PF.case_inputs(seed, N, K, B, entry, kw, y0, extra)
    return seed, {e: _PF.floor_parts(N, K, ins, e, dense_once=True) for e in envs}


def floor_of(parts, kind):
    """"three": the floor of DESIGN.md 4 (max of the AMD and dense-LU distances); "dense": round 5's
    (the dense-LU distance alone), reported beside it."""
    return parts["dense"] if kind == "dense" else [max(a, b) for a, b in zip(parts["dense"], parts["amd"])]


def passes(rec, fl, tol):
    """rec = [env, ex, es, ez, ey, eu]: within max(bound, 4x floor) in every output."""
    errs = rec[1:]
    ok = all(errs[k] <= max(tol, 4.0 * fl[k]) for k in range(4)) and errs[4] <= max(1e-4, 4.0 * fl[4])
    ratio = max([errs[k] / max(fl[k], 1e-300) for k in range(4) if errs[k] > tol] +
                [errs[4] / max(fl[4], 1e-300)] * (errs[4] > 1e-4) + [0.0])
    return ok, ratio


def main():
    src = sys.argv[1]
    out_path = sys.argv[2] if len(sys.argv) > 2 else src.replace(".json.gz", "") + ".floor.json"
    camp = json.load(gzip.open(src, "rt"))
    summ, cases = camp["summary"], [c for c in camp["cases"] if "oracle_failed" not in c]
    ccs = bool(summ.get("ccs"))
    policies, full = summ["policies"], set(summ.get("full_record", []))
    max_fails = int(os.environ.get("FLOOR_MAX_FAILS", "200"))
    seq = "ccs" if ccs else "default"
    cache_path = os.environ.get("FLOOR_CACHE", os.path.join(ROOT, "profiles", "r06", f"floor_cache_{seq}.json.gz"))
    cache = json.load(gzip.open(cache_path, "rt")) if os.path.exists(cache_path) else {}
    _init(ccs, {})
    params = _PF.replay_all(max(c["seed"] for c in cases))
    by_seed = {c["seed"]: c for c in cases}
    t0 = time.time()

    # per (policy, case): the recorded envs and a cursor
    state = {}
    for p in policies:
        for c in cases:
            col = c["cols"][p]
            if "same_as" in col:
                continue
            state[(p, c["seed"])] = {"recs": col["above"], "i": 0, "fails": [], "worst": 0.0,
                                     "finite": col["finite"], "done": False}
    nfail = {p: 0 for p in policies}
    with Pool(int(os.environ.get("FLOOR_WORKERS", "8")), initializer=_init, initargs=(ccs, params)) as pool:
        while True:
            need = {}
            for (p, seed), st in state.items():
                if st["done"]:
                    continue
                if p not in full and nfail[p] >= max_fails:
                    st["done"], st["unverified"] = True, True
                    continue
                recs, i = st["recs"], st["i"]
                # every pending env of a full-record policy at once; the next one otherwise
                want = recs[i:] if p in full else recs[i:i + 1]
                for r in want:
                    if f"{seed}:{r[0]}" not in cache:
                        need.setdefault(seed, set()).add(r[0])
            if need:
                tasks = sorted(((s, sorted(v)) for s, v in need.items()), key=lambda t: -by_seed[t[0]]["N"] ** 3 * len(t[1]))
                for seed, fl in pool.imap_unordered(floors_of, tasks):
                    for e, v in fl.items():
                        cache[f"{seed}:{e}"] = v
                print(json.dumps({"floors_computed": sum(len(v) for v in need.values()), "cache": len(cache),
                                  "s": round(time.time() - t0, 1)}), flush=True)
            progressed = False
            for (p, seed), st in state.items():
                if st["done"]:
                    continue
                tol = by_seed[seed]["tol"]
                while st["i"] < len(st["recs"]):
                    rec = st["recs"][st["i"]]
                    fl = cache.get(f"{seed}:{rec[0]}")
                    if fl is None:
                        break
                    ok_d, _ = passes(rec, floor_of(fl, "dense"), tol)
                    st["fails_dense"] = st.get("fails_dense", 0) + (not ok_d)
                    fl = floor_of(fl, "three")
                    ok, ratio = passes(rec, fl, tol)
                    st["worst"] = max(st["worst"], ratio)
                    st["i"] += 1
                    progressed = True
                    if not ok:
                        st["fails"].append({"env": rec[0], "err": rec[1:], "floor": fl, "ratio": ratio})
                        if p not in full:
                            break
                if st["fails"] and (p not in full or st["i"] >= len(st["recs"])):
                    st["done"] = True
                    nfail[p] += 1
                elif st["i"] >= len(st["recs"]):
                    st["done"] = True
            if not need and not progressed:
                break
    os.makedirs(os.path.dirname(cache_path), exist_ok=True)
    with gzip.open(cache_path, "wt") as fh:
        json.dump(cache, fh)

    report = {"campaign": os.path.basename(src), "build_id": summ.get("build_id"), "ccs": ccs,
              "cases": len(cases), "envs": int(sum(c["B"] for c in cases)), "floor_seconds": round(time.time() - t0, 1),
              "floor": "max(|AMD LDL^T - MD LDL^T|, |dense LU - MD LDL^T|) per output, relative per env",
              "floor_dense_only": "failed_cases_dense_floor_only: the same check against |dense LU - MD LDL^T| "
                                  "alone (round 5's floor; for a policy outside the full-record set a lower "
                                  "bound: its cases stop at the first env failing the three-way floor)",
              "policies": {}}
    for p in policies:
        failed, unverified, recorded, unchecked, not_recorded, big, worst = [], 0, 0, 0, 0, 0, 0.0
        failed_dense = 0
        max_x = max_u0 = 0.0
        for c in cases:
            col = c["cols"][p]
            base = p if "same_as" not in col else col["same_as"]
            bcol = c["cols"][base]
            st = state[(base, c["seed"])]
            recorded += len(bcol["above"])
            not_recorded += bcol["n_above"] - len(bcol["above"])
            unchecked += len(bcol["above"]) - st["i"] + (bcol["n_above"] - len(bcol["above"]))
            max_x, max_u0 = max(max_x, bcol["max_err"]), max(max_u0, bcol["max_u0_rel"])
            if st.get("unverified"):
                unverified += 1
                continue
            bad = st["fails"] or not st["finite"]
            failed_dense += bool(st.get("fails_dense", 0) or not st["finite"])
            for f in st["fails"]:  # over 1e-4 in x or u0 AND beyond 4x the floor in that same output
                big += any(f["err"][k] > max(1e-4, 4.0 * f["floor"][k]) for k in (0, 4))
            if bad:
                worst = max(worst, max(f["ratio"] for f in st["fails"]) if st["fails"] else float("inf"))
                failed.append({k: c[k] for k in ("seed", "N", "K", "B", "entry", "K0", "path", "y0")} |
                              {"n_above": bcol["n_above"], "fails": st["fails"][:4], "finite": st["finite"]})
        report["policies"][p] = {
            "failed_cases": len(failed), "worst_ratio_to_floor": worst,
            "failed_cases_dense_floor_only": failed_dense, "unverified_cases": unverified,
            "above_tol_envs_recorded": recorded, "above_tol_unchecked_envs": unchecked,
            "above_tol_not_recorded": not_recorded,
            "envs_over_1e-4_in_x_or_u0_beyond_4x_floor": big,
            "max_err_any_output": max_x, "max_u0_rel": max_u0,
            "by_path": {k: sum(f["path"] == k for f in failed) for k in ("auto", "lds", "general")},
            "fully_checked": bool(unverified == 0 and unchecked == 0),
            "failed": failed}
        print(json.dumps({"policy": p} | {k: v for k, v in report["policies"][p].items() if k != "failed"}), flush=True)
    with open(out_path, "w") as fh:
        json.dump(report, fh, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
