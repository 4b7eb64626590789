"""Randomised parity campaign on the GPU box: HIP path vs the oracle over random configurations.

    python scripts/parity_fuzz.py [SECONDS] [OUT_JSON_GZ]     (default 150 s, gpurun_out/parity_fuzz.json.gz)
    FUZZ_CASES=n: exactly the first n cases of the fixed random sequence instead of a time budget
    SRBD_LIB=path: another build of libsrbd_mpc.so (A/B of two libraries on the same cases)
    FUZZ_POLICIES=name,...: the refinement policies to run every case under (POLICIES below; default
      "adaptive,strict", the two srbd_set_refinement modes); FUZZ_REFINE=mode: that mode alone (round 5)
    FUZZ_CCS=1: adds the reference's _ccs entry to the draw (a different random sequence)
    FUZZ_SEEDS=s1,s2,...: exactly those cases of the sequence (replayed); FUZZ_FULL / FUZZ_CAP_OTHER: below
    FUZZ_ROWS=1: also the HIP x, s, z, y rows of every recorded env of the full-record policies, in
      OUT_JSON_GZ's name + .rows.npz (keys "<policy>/<seed>/<env>/<x|s|z|y>"; large: for replays of chosen seeds)

Each case draws a horizon N in 1..32, an iteration count K in 1..25, a batch B in 1..300, an entry
(fused step with y0 in {0, 1}; the solver from the GPU caller's cold init; the solver warm-started
from the oracle's iterate after K0 iterations -- the reference caller's chained calls; with FUZZ_CCS=1
also the reference's _ccs entry from a random x_init), a solver path (auto / lds / general) and a
workload (SURVEY 8d distributions with random tilt, residual scale, randomized gait or a random flight /
single-support override), computes the oracle once, runs the HIP call under every policy through the
C-ABI (the policies act on the register kernels only: a case on the lds or general path, or at N = 1,
runs once and its result stands for every policy), and records, per policy, EVERY env outside
  * u0 (the controller's output) within 1e-4 relative (north_star), or
  * x, s, z, y within the parity tests' tolerance for K (1e-10 / 1e-9 / 1e-7 / 1e-5 at K <= 1 / 5 / 10 /
    more)
with its five errors. Such an env passes only within 4x its own FP64 floor -- the spread of the CPU
restatements on that env -- which is computed offline on the CPU host, for every recorded env, by
scripts/parity_floor.py (a case is "ok" only when every recorded env of it has been floor-checked and
passed). Policies outside FUZZ_FULL (default: the two modes) record at most FUZZ_CAP_OTHER = 32 envs per
case (their worst), enough to reject a variant; the modes record all.
Test infrastructure: the oracle is the checker only.
"""
import gzip
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from biped_pympc_amd import _native, solver  # noqa: E402
from biped_pympc_amd.utils.synthetic import make_workload, solver_init  # noqa: E402
from oracle import oracle  # noqa: E402
from tests._util import rel_err_rows  # noqa: E402

# FUZZ_CCS=1 adds the reference's _ccs entry (x from x_init, s = max(h - G x, 1), z = 1, y = 0;
# srbd_pdipm_ccs) to the draw -- a different random sequence from the default one, which
# tests/golden/make_fuzz_regressions.py replays
ENTRIES = ["fused", "cold", "warm"] + (["ccs"] if os.environ.get("FUZZ_CCS") == "1" else [])

_F = _native.refine_affine_first
_L = _native.refine_affine_last
# name -> ("mode", srbd_set_refinement mode) or (srbd_set_refinement_policy flags, W threshold[, alpha])
POLICIES = {
    "adaptive": ("mode", 0),            # the default: affine refined at the initial iterate (all z = 1), W >= 1e4, clamp
    "strict": ("mode", 1),              # the affine direction refined in every iteration
    "w1e3": (0, 1e3),                   # round 5's mode 0: W >= 1e3 / clamp only
    "init_w1e3": (2, 1e3),
    "init_w2e3": (2, 2e3),
    "init_w3e3": (2, 3e3),
    "init_w5e3": (2, 5e3),
    "init_w1e4": (2, 1e4),              # = mode 0 since round 6
    "init_w3e4": (2, 3e4),
    "init_only": (2, 0.0),              # the initial-iterate vote alone (w <= 0: no W vote; clamps still vote)
    "w5e3": (0, 5e3),
    "first1": (_F(1), 1e3),             # the first iteration of every call (position-based)
    "first2": (_F(2), 1e3),
    "first1_last1": (_F(1) | _L(1), 1e3),
    "w1e2": (0, 1e2),
    "w1e4": (0, 1e4),
    "first1_w1e2": (_F(1), 1e2),
    "first1_w3e2": (_F(1), 3e2),
    "first1_w3e3": (_F(1), 3e3),
    "first1_w1e4": (_F(1), 1e4),
}
# Measured in round 6 on builds of their own (profiles/r06/), rejected: the combined direction
# unrefined, refined in the last ceil(K / 2) iterations only, or in its dual rows only (SRBD_REFINE_COMBINED =
# 1 / 2 / 3), and a trigger on the previous combined step length
FULL = set(os.environ.get("FUZZ_FULL", "adaptive,strict").split(","))
CAP_OTHER = int(os.environ.get("FUZZ_CAP_OTHER", "32"))


def policy_ctx(name):
    kind, *v = POLICIES[name]
    return _native.refinement(("adaptive", "every_iteration")[v[0]]) if kind == "mode" else \
        _native.refinement_policy(kind, *v)


def floor_parts(N, K, ins, e, dense_once=False):
    """Env e's distances from the checker (the sparse LDL^T under exact minimum degree) of the two other CPU
    restatements, per output x, s, z, y and the u0 slice, relative per env: {"dense": dense LU
    (oracle/pdipm_dense.py), "amd": the same LDL^T under AMD, the ordering of the reference's ca.ldl
    (sparse_pdipm_solver.py:451)}."""
    from oracle.pdipm_dense import pdipm_dense
    one = [np.asarray(a)[e:e + 1] for a in ins]
    md = oracle.pdipm(N, K, one, nthreads=1)
    am = oracle.pdipm(N, K, one, nthreads=1, order="amd")
    dn = pdipm_dense(N, K, *[a[0] for a in one], factor_once=dense_once)
    dn = [np.asarray(v)[None] for v in dn[:4]]
    u = slice(12 * N, 12 * N + 12)

    def dist(o):
        return [float(rel_err_rows(o[k], md[k]).max()) for k in range(4)] + \
               [float(rel_err_rows(o[0][:, u], md[0][:, u]).max())]
    return {"dense": dist(dn), "amd": dist(am)}


def floor_env(N, K, ins, e, dense_once=False):
    """The FP64 floor of env e: per output, the larger of floor_parts' two distances."""
    fp = floor_parts(N, K, ins, e, dense_once)
    return [max(a, b) for a, b in zip(fp["dense"], fp["amd"])]


def tol_for(K):
    return 1e-10 if K <= 1 else 1e-9 if K <= 5 else 1e-7 if K <= 10 else 1e-5


def cuda(arrs):
    return [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in arrs]


def draw(rng):
    N = int(rng.integers(1, 33))
    K = int(rng.integers(1, 26))
    B = int(rng.integers(1, 301))
    entry = str(rng.choice(ENTRIES))
    path = str(rng.choice(["auto", "auto", "lds", "general"]))
    kw = dict(tilt=float(rng.uniform(0.0, 0.5)), residuals=bool(rng.integers(0, 2)),
              residual_scale=float(rng.uniform(0.1, 2.0)), random_gait=bool(rng.integers(0, 2)))
    if rng.random() < 0.2:  # a contact override: flight or single support over the whole horizon
        c = np.zeros((B, N, 2), np.int32)
        c[:, :, 0] = int(rng.integers(0, 2))
        c[:, :, 1] = int(rng.integers(0, 2))
        kw["contact_override"] = c
        kw["random_gait"] = False
    y0 = float(rng.integers(0, 2))
    return N, K, B, entry, path, kw, y0


def draw_case(rng):
    """draw() plus the entry's own draws, in the order the campaign consumes the generator."""
    N, K, B, entry, path, kw, y0 = draw(rng)
    extra = {}
    if entry == "ccs":
        extra["scale"] = float(rng.uniform(0.1, 5.0))
    elif entry == "warm":
        extra["K0"] = int(rng.integers(1, 11))
    return N, K, B, entry, path, kw, y0, extra


def replay(seed_want):
    """The campaign's case `seed_want` (seeds count from 50000 in draw order)."""
    rng = np.random.default_rng(20261018)
    for seed in range(50000, seed_want + 1):
        case = draw_case(rng)
    return case


def replay_all(seed_max):
    """{seed: case} for every seed up to seed_max, in one pass over the generator."""
    rng = np.random.default_rng(20261018)
    return {seed: draw_case(rng) for seed in range(50000, seed_max + 1)}


def case_inputs(seed, N, K, B, entry, kw, y0, extra):
    """The case's workload and solver inputs [H, G, A, f, d, b, x, s, z, y] (the start of its iterations)."""
    wl = make_workload(B, N, seed=seed, **kw)
    H, f, A, b, G, d = oracle.qp_former(N, wl.inputs)
    if entry == "ccs":
        from biped_pympc_amd import layout
        dims = layout.Dims(N)
        x0 = np.random.default_rng(seed).normal(0.0, extra["scale"], (B, dims.nz))
        Gd = layout.to_dense(G, *layout.ccs_G(N), (dims.n_ineq, dims.nz))
        s0 = np.maximum(d - np.einsum("bij,bj->bi", Gd, x0), 1.0)
        it = [x0, s0, np.ones((B, dims.n_ineq)), np.zeros((B, dims.n_eq))]
    else:
        it = list(solver_init(d, N, y0))
        if entry == "warm":
            it = oracle.pdipm(N, extra["K0"], [H, G, A, f, d, b, *it])[:4]
    return wl, [H, G, A, f, d, b, *it]


def hip_solve(N, K, entry, path, y0, wl, ins, policy):
    """The case's HIP call: fused step, srbd_pdipm_ccs, or srbd_pdipm from the given iterate."""
    with _native.solver_path(path), policy_ctx(policy):
        if entry == "fused":
            return solver.mpc_solve(cuda(wl.inputs), N, K, y0=y0)
        if entry == "ccs":
            return solver.pdipm_ccs(cuda(ins[:6]), cuda([ins[6]])[0], N, K)
        return solver.pdipm(cuda(ins[:6]), cuda(ins[6:]), N, K)


def env_errors(got, ref, N):
    """(B, 5): x, s, z, y relative errors per env and the u0 slice's."""
    errs = np.stack([rel_err_rows(got[k], ref[k]) for k in range(4)], 1)
    u = slice(12 * N, 12 * N + 12)
    return np.concatenate([errs, rel_err_rows(got[0][:, u], ref[0][:, u])[:, None]], 1)


def score(errs, tol):
    """How far past its bound each env is (> 1: outside the tolerance or the u0 bound)."""
    return np.maximum((errs[:, :4] / tol).max(1), errs[:, 4] / 1e-4)


ROWS = {}  # FUZZ_ROWS=1: "<policy>/<seed>/<env>/<x|s|z|y>" -> the HIP row


def run_case(seed, rng, policies):
    N, K, B, entry, path, kw, y0, extra = draw_case(rng)
    wl, ins = case_inputs(seed, N, K, B, entry, kw, y0, extra)
    ref = oracle.mpc_solve(N, K, wl.inputs, y0=y0) if entry == "fused" else oracle.pdipm(N, K, ins)
    tol = tol_for(K)
    cols, first = {}, None
    sensitive = path == "auto" and N >= 2  # the register kernels: the policies act there only
    for pol in policies:
        if first is not None and not sensitive:
            cols[pol] = {"same_as": first}
            continue
        got = hip_solve(N, K, entry, path, y0, wl, ins, pol)
        torch.cuda.synchronize()
        got = [t.cpu().numpy() for t in got]
        errs = env_errors(got, ref, N)
        sc = score(errs, tol)
        above = np.flatnonzero(sc > 1.0)
        above = above[np.argsort(-sc[above])]
        cap = len(above) if pol in FULL else CAP_OTHER
        if os.environ.get("FUZZ_ROWS") == "1" and pol in FULL:
            for e in above:
                for k, v in enumerate("xszy"):
                    ROWS[f"{pol}/{seed}/{int(e)}/{v}"] = got[k][e].copy()
        cols[pol] = {"max_err": float(errs[:, :4].max()), "max_u0_rel": float(errs[:, 4].max()),
                     "n_above": int(len(above)),
                     "above": [[int(e)] + [float(f"{v:.4g}") for v in errs[e]] for e in above[:cap]],
                     "finite": bool(all(np.all(np.isfinite(g)) for g in got))}
        first = first or pol
    return {"seed": seed, "N": N, "K": K, "B": B, "entry": entry, "K0": extra.get("K0", 0), "path": path,
            "y0": y0, "tilt": round(kw["tilt"], 3), "residuals": kw["residuals"],
            "random_gait": kw["random_gait"], "override": "contact_override" in kw, "tol": tol, "cols": cols}


def main():
    budget = float(sys.argv[1]) if len(sys.argv) > 1 else 150.0
    out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out", "parity_fuzz.json.gz")
    if os.environ.get("FUZZ_REFINE"):
        policies = [{"every_iteration": "strict"}.get(os.environ["FUZZ_REFINE"], "adaptive")]
    else:
        policies = os.environ.get("FUZZ_POLICIES", "adaptive,strict").split(",")
    for p in policies:
        assert p in POLICIES, p
    rng = np.random.default_rng(20261018)
    t0, cases = time.time(), []
    seed = 50000
    max_cases = int(os.environ.get("FUZZ_CASES", "0"))  # a fixed case list (A/B of two libraries)
    # FUZZ_SEEDS=s1,s2,...: exactly those cases of the sequence (replayed; regression fixtures)
    only = sorted(int(v) for v in os.environ.get("FUZZ_SEEDS", "").split(",") if v)
    if only:
        max_cases = only[-1] - 50000 + 1
    while (len(cases) < max_cases) if max_cases else (time.time() - t0 < budget):
        if only and seed not in only:
            draw_case(rng)
            seed += 1
            continue
        try:
            c = run_case(seed, rng, policies)
        except FloatingPointError as ex:  # the checker's own LDL failed (oracle status): no verdict
            c = {"seed": seed, "oracle_failed": str(ex), "B": 0, "N": 0, "K": 0, "entry": "-", "path": "-",
                 "cols": {}}
        cases.append(c)
        if only and seed == only[-1]:
            max_cases = len(cases)
        brief = {p: (v.get("n_above"), f"{v['max_u0_rel']:.1e}") for p, v in c["cols"].items() if "n_above" in v}
        print(json.dumps({k: c[k] for k in ("seed", "N", "K", "B", "entry", "path")} | {"above": brief}), flush=True)
        seed += 1
    summary = {
        "cases": len(cases), "envs": int(sum(c["B"] for c in cases)), "policies": policies,
        "policy_words": {p: POLICIES[p] for p in policies}, "full_record": sorted(FULL & set(policies)),
        "oracle_failed_cases": int(sum("oracle_failed" in c for c in cases)),
        "horizons": sorted({c["N"] for c in cases if c["N"]}), "iterations": sorted({c["K"] for c in cases if c["K"]}),
        "by_entry": {e: sum(c["entry"] == e for c in cases) for e in ENTRIES},
        "by_path": {p: sum(c["path"] == p for c in cases) for p in ("auto", "lds", "general")},
        "seconds": round(time.time() - t0, 1), "build_id": _native.build_id(), "ccs": "ccs" in ENTRIES,
    }
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with gzip.open(out, "wt") as fh:
        json.dump({"summary": summary, "cases": cases}, fh)
    if ROWS:
        np.savez_compressed(out.replace(".json.gz", "") + ".rows.npz", **ROWS)
    print(json.dumps(summary))
    return 0


if __name__ == "__main__":
    sys.exit(main())
