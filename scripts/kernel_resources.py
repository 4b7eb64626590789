"""Per-kernel register / spill / scratch figures from a hipcc -S listing (the AMDGPU metadata).

    python scripts/kernel_resources.py /tmp/main.s [substring]
    python scripts/kernel_resources.py --table > profiles/rNN/kernel_resources.txt
        (compiles every product unit to device ISA with the product flags, srbd_regN.hip in its six
        horizon parts, and prints one row per kernel)
"""
import re
import sys


def resources(path, want=""):
    text = open(path).read()
    out = {}
    for block in re.split(r"\n\s+- \.", text.split("amdhsa.kernels:")[-1]):
        name = re.search(r"\.name:\s+(\S+)", block)
        if not name or want not in name.group(1):
            continue
        get = lambda k: int(re.search(rf"\.{k}:\s+(\d+)", block).group(1)) if re.search(rf"\.{k}:\s+(\d+)", block) else None
        out[name.group(1)] = {k: get(k) for k in ("vgpr_count", "agpr_count", "vgpr_spill_count", "sgpr_spill_count",
                                                  "private_segment_fixed_size", "group_segment_fixed_size")}
    return out


# instructions of a call's whole-wave register save / restore sequence (the SGPR-spill lanes written or
# read around it, exec toggles, waits, the other saves), which may sit between a spill and its call
_CALL_SEQ = ("v_writelane_b32", "v_readlane_b32", "s_nop", "s_or_saveexec_b64", "s_mov_b64 exec",
             "s_waitcnt", "scratch_store_dword", "scratch_load_dword", "; implicit-def",
             "v_mov_b32_e32 v0,", "v_mov_b32_e32 v1,", "v_mov_b64_e32 v[0:1],")  # (the call's return value)


def _call_adjacent(body, i, step, calls):
    j = i + step
    while 0 <= j < len(body):
        if j in calls:
            return True
        t = body[j].strip()
        if not t or not t.startswith(_CALL_SEQ):
            return False
        j += step
    return False


def body_spills(path, kernel):
    """VGPR spill / reload instructions of `kernel` (mangled name) outside the save / restore sequence of
    a call: a spill followed by an s_swappc_b64, or a reload preceded by one, with nothing but that
    sequence's own instructions in between (_CALL_SEQ) is the caller keeping a register across the call
    (the in-launch fallback's: the whole-wave SGPR-spill registers it must save around any call) and runs
    only on that path. Returns the other lines."""
    body, on = [], False
    for line in open(path):
        if line.startswith(kernel + ":"):
            on = True
        elif on and line.startswith(".Lfunc_end"):
            break
        if on:
            body.append(line.rstrip("\n"))
    calls = {i for i, l in enumerate(body) if "s_swappc_b64" in l}
    out = []
    for i, l in enumerate(body):
        if "Folded Spill" in l and not _call_adjacent(body, i, 1, calls):
            out.append(l.strip())
        elif "Folded Reload" in l and not _call_adjacent(body, i, -1, calls):
            out.append(l.strip())
    return out


def table(tmpdir="/tmp/kernel_resources"):
    """The kernel_resources.txt table of every product translation unit (product flags)."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    from biped_pympc_amd.build import HIP_UNITS, source_hash, unit_compile_cmd
    os.makedirs(tmpdir, exist_ok=True)
    jobs = []
    for unit in HIP_UNITS:
        parts = [[f"-DSRBD_REGN_PART={k}"] for k in range(6)] if unit == "srbd_regN.hip" else [[]]
        for k, defs in enumerate(parts):
            out = os.path.join(tmpdir, f"{unit}.{k}.s")
            tag = f"{unit}/{k}" if len(parts) > 1 else unit
            cmd = unit_compile_cmd(unit, [*defs, "--cuda-device-only", "-S", "-o", out])
            jobs.append((tag, out, subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)))
    rows = []
    for tag, out, p in jobs:
        err = p.communicate()[1]
        if p.returncode:
            raise SystemExit(err.decode()[-2000:])
        for name, r in resources(out).items():
            dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
            dem = re.sub(r"\(.*\)$", "", dem)
            rows.append((tag, dem, r))
    print(f"# Per-kernel resources from the gfx950 device ISA (hipcc --cuda-device-only -S, product flags;\n"
          f"# scripts/kernel_resources.py --table). Sources at build id {source_hash()}. vgpr = arch VGPRs, spill =\n"
          f"# VGPR spills as the compiler reports them (the CCS kernels' one or two: the whole-wave save around the\n"
          f"# fallback call, see tests/test_isa_hazards.py), scratch = private segment bytes per lane (call stack),\n"
          f"# lds = static LDS.")
    print(f"{'unit':18s} {'kernel':52s} {'vgpr':>4s} {'agpr':>4s} {'spill':>5s} {'sgpr_spill':>10s} {'scratch':>7s} {'lds':>5s}")
    fmt = lambda v: "-" if v is None else str(v)
    for tag, dem, r in rows:
        print(f"{tag:18s} {dem[:52]:52s} {fmt(r['vgpr_count']):>4s} {fmt(r['agpr_count']):>4s} "
              f"{fmt(r['vgpr_spill_count']):>5s} {fmt(r['sgpr_spill_count']):>10s} "
              f"{fmt(r['private_segment_fixed_size']):>7s} {fmt(r['group_segment_fixed_size']):>5s}")


if __name__ == "__main__":
    if sys.argv[1:] == ["--table"]:
        table()
        sys.exit(0)
    for n, r in resources(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "").items():
        print(f"{n[:60]:60s} " + " ".join(f"{k}={v}" for k, v in r.items()))
