"""The parity campaign's offline floor check (scripts/parity_floor.py; CPU only, test infrastructure).

A campaign (scripts/parity_fuzz.py, on the GPU box) records every env outside its bounds; the floor check
decides each case. These tests fabricate a two-policy campaign over real cases of the default sequence
(small horizons, so the floors take seconds) with errors placed relative to each env's own floor, and check
the verdicts: an env within 4x its floor passes, one beyond fails its case, a full-record policy checks every
recorded env even after a failure (no unchecked env), another policy stops at its first failing env, and a
case whose column points at another policy's ("same_as": the lds / general paths, N = 1) takes that verdict.
"""
import gzip
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SEEDS = (50003, 50004)  # default sequence: N = 4, K = 15, B = 43, cold, auto; N = 1, K = 15, B = 212, fused


@pytest.fixture(scope="module")
def pf():
    os.environ["FUZZ_CCS"] = "0"
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import importlib
    mod = importlib.import_module("parity_fuzz")
    assert "ccs" not in mod.ENTRIES
    return mod


def test_replay_all_matches_replay(pf):
    allc = pf.replay_all(50010)
    for seed in (50000, 50004, 50010):
        a, b = allc[seed], pf.replay(seed)
        assert a[:5] == b[:5] and a[6:] == b[6:]
    assert allc[50003][:5] == (4, 15, 43, "cold", "auto") and allc[50004][:5] == (1, 15, 212, "fused", "auto")


def test_floor_check_verdicts(pf, tmp_path):
    params = pf.replay_all(max(SEEDS))
    cases = []
    for seed in SEEDS:
        N, K, B, entry, path, kw, y0, extra = params[seed]
        _, ins = pf.case_inputs(seed, N, K, B, entry, kw, y0, extra)
        tol = pf.tol_for(K)
        fl = [pf.floor_env(N, K, ins, e, dense_once=True) for e in (0, 1)]
        # env 0 within 4x its floor in z (and above the tolerance), env 1 at 10x its floor in x
        ok_rec = [0, 0.0, 0.0, max(2.0 * fl[0][2], 1.5 * tol), 0.0, 0.0]
        bad_rec = [1, max(10.0 * fl[1][0], 10.0 * tol), 0.0, 0.0, 0.0, 0.0]
        if max(2.0 * fl[0][2], 1.5 * tol) > 4.0 * fl[0][2]:  # a tiny floor: env 0 would not pass by it
            ok_rec[3] = 0.0
        recs = [bad_rec, ok_rec] if seed == SEEDS[0] else [ok_rec]
        cols = {"full": {"max_err": 1.0, "max_u0_rel": 0.0, "n_above": len(recs), "above": recs, "finite": True},
                "other": ({"max_err": 1.0, "max_u0_rel": 0.0, "n_above": 2, "above": [bad_rec, ok_rec], "finite": True}
                          if seed == SEEDS[0] else {"same_as": "full"})}
        cases.append({"seed": seed, "N": N, "K": K, "B": B, "entry": entry, "K0": extra.get("K0", 0), "path": path,
                      "y0": y0, "tol": tol, "cols": cols})
    camp = tmp_path / "camp.json.gz"
    with gzip.open(camp, "wt") as fh:
        json.dump({"summary": {"policies": ["full", "other"], "full_record": ["full"], "ccs": False, "build_id": "t"},
                   "cases": cases}, fh)
    out = tmp_path / "camp.floor.json"
    env = dict(os.environ, FLOOR_WORKERS="2", FLOOR_CACHE=str(tmp_path / "cache.json.gz"))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "parity_floor.py"), str(camp), str(out)],
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    rep = json.load(open(out))
    full, other = rep["policies"]["full"], rep["policies"]["other"]
    # seed 1 fails (env 1 at 10x its floor), seed 2 passes
    assert full["failed_cases"] == 1 and [c["seed"] for c in full["failed"]] == [SEEDS[0]]
    assert full["above_tol_unchecked_envs"] == 0 and full["fully_checked"]
    assert full["failed"][0]["fails"][0]["env"] == 1 and full["failed"][0]["fails"][0]["ratio"] >= 9.9
    # the other policy stops at its first failing env (its env 0 stays unchecked) and takes seed 2's
    # verdict from "full"
    assert other["failed_cases"] == 1 and other["above_tol_unchecked_envs"] == 1 and not other["fully_checked"]
    assert os.path.exists(tmp_path / "cache.json.gz")
