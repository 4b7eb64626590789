"""Per-kernel register / spill / scratch figures from a hipcc -S listing (the AMDGPU metadata).

    python scripts/kernel_resources.py /tmp/main.s [substring]
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


def body_spills(path, kernel, window=12):
    """VGPR spill / reload instructions of `kernel` (mangled name) outside the save / restore sequence of
    a call: a spill followed by an s_swappc_b64 within `window` lines, or a reload preceded by one, is
    the caller keeping a register across the call (the in-launch fallback's: the whole-wave SGPR-spill
    register it must save around any call) and runs only on that path. Returns the other lines."""
    body, on = [], False
    for line in open(path):
        if line.startswith(kernel + ":"):
            on = True
        elif on and line.startswith(".Lfunc_end"):
            break
        if on:
            body.append(line.rstrip("\n"))
    calls = [i for i, l in enumerate(body) if "s_swappc_b64" in l]
    out = []
    for i, l in enumerate(body):
        if "Folded Spill" in l and not any(0 < j - i <= window for j in calls):
            out.append(l.strip())
        elif "Folded Reload" in l and not any(0 < i - j <= window for j in calls):
            out.append(l.strip())
    return out


if __name__ == "__main__":
    for n, r in resources(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "").items():
        print(f"{n[:60]:60s} " + " ".join(f"{k}={v}" for k, v in r.items()))
