"""Static instruction mix per solver phase of the fused N=10 kernel (diagnostic, CPU only).

python scripts/isa_phase_mix.py [--top K] [extra hipcc flags...]

Builds the fused kernel with scripts/phase_prof.hpp force-included (s_memtime stamps at the phase boundaries, see
srbd_common.hpp), splits the kernel's ISA at the stamps and counts instruction classes per
segment: FP64 arithmetic, the inline-asm broadcast-FMAs, 32-bit integer/compare/select work
(address and predicate arithmetic), moves, LDS and scalar instructions. Static counts of straight-
line code equal per-iteration dynamic counts up to exec-skipped branches and the rolled loops.
"""
import os
import re
import subprocess
import sys

ROOT = __file__.rsplit("/scripts/", 1)[0]
SYM = "_ZN4srbd19mpc_step_reg_kernelILi10EEEvNS_9FusedArgsE"
CLASSES = [
    ("dppfma", r"v_fmac_f64_dpp"),
    ("f64", r"v_(fma|fmac|mul|add|max|min|rcp|ldexp|div_\w+|frexp\w*|sqrt|rsq|cmp_\w+)_f64"),
    ("int", r"v_(add|sub|subrev|mul_lo|mul_hi|mad_\w+|lshl\w*|lshr\w*|ashr\w*|and|or|xor|min_[iu]\d+|max_[iu]\d+|"
            r"bfe\w*|add3|addc\w*|subb\w*|cmp\w*|cndmask|readlane|readfirstlane|mul_u32\w*|mul_i32\w*|not|bfi|alignbit|perm)"),
    ("mov", r"v_mov"),
    ("lds", r"ds_"),
    ("vmem", r"(global|buffer|flat)_"),
    ("salu", r"s_"),
]


def main():
    top = 0
    if len(sys.argv) > 2 and sys.argv[1] == "--top":
        top = int(sys.argv[2])
        del sys.argv[1:3]
    out = "/tmp/isa_phase_mix.s"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", f"-I{ROOT}/include",
                    "--cuda-device-only", "-S", "-include", os.path.join(ROOT, "scripts", "phase_prof.hpp"), *sys.argv[1:], "-o", out,
                    f"{ROOT}/biped_pympc_amd/csrc/srbd_mpc.hip"], check=True, stderr=subprocess.DEVNULL)
    lines, on = [], False
    for ln in open(out):
        if ln.startswith(SYM + ":"):
            on = True
        if on:
            lines.append(ln)
            if "s_endpgm" in ln:
                break
    segs, cur = [], []
    for ln in lines:
        s = ln.strip()
        if s.startswith("s_memtime"):
            segs.append(cur)
            cur = []
        elif s and not s.startswith((";", ".")):
            cur.append(s.split()[0])
    segs.append(cur)
    print(f"{'seg':>4} {'total':>6} " + " ".join(f"{c:>7}" for c, _ in CLASSES) + "  other")
    for k, seg in enumerate(segs):
        cnt = {c: 0 for c, _ in CLASSES}
        other = 0
        for op in seg:
            for c, pat in CLASSES:
                if re.match(pat, op):
                    cnt[c] += 1
                    break
            else:
                other += 1
        print(f"{k:>4} {len(seg):>6} " + " ".join(f"{cnt[c]:>7}" for c, _ in CLASSES) + f"  {other}")
        if top:  # the segment's most frequent non-FP64 vector instructions
            hist = {}
            for op in seg:
                if op.startswith("v_") and not re.match(CLASSES[0][1] + "|" + CLASSES[1][1], op):
                    hist[op] = hist.get(op, 0) + 1
            print("       " + ", ".join(f"{o} {n}" for o, n in sorted(hist.items(), key=lambda x: -x[1])[:top]))


if __name__ == "__main__":
    main()
