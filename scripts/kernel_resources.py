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


if __name__ == "__main__":
    for n, r in resources(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "").items():
        print(f"{n[:60]:60s} " + " ".join(f"{k}={v}" for k, v in r.items()))
