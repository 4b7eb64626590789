"""Static check of the VALU-write -> DPP-read hazard (2 wait states) in a kernel's ISA, inline asm
included: for every DPP instruction, the instructions issued in the 2 wait states before it must not
write ANY VGPR it reads -- the DPP-routed src0, the other sources and, for v_fmac/v_mac, the
accumulator (src2 = vdst). That is LLVM's GCNHazardRecognizer rule (every VGPR use of a DPP
instruction), which the asm blocks cannot rely on the compiler to enforce. s_nop N counts N + 1
states, other instructions 1. The scan walks back along every control-flow predecessor: the
fall-through instruction (unless it is an unconditional s_branch / s_endpgm / s_setpc) and every
branch that targets a label it crosses.

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -DSRBD_SPLIT_REG20 --cuda-device-only -S \
        -o /tmp/k.s biped_pympc_amd/csrc/srbd_mpc.hip
    python scripts/dpp_hazard_check.py /tmp/k.s [kernel-symbol-substring]
"""
import re
import sys

REG = re.compile(r"\bv(\d+)\b|\bv\[(\d+):(\d+)\]")
BRANCH = re.compile(r"^s_(c?branch\w*|cbranch\w*)\s+(\S+)")
NOFALL = ("s_branch", "s_endpgm", "s_setpc_b64")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(1) is not None:
            out.add(int(m.group(1)))
        else:
            out.update(range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def parse(lines):
    """(kind, dst_regs, src_regs, text, states, op, label) per line; kind: 'label', 'inst', 'skip'."""
    out = []
    for raw in lines:
        s = raw.split(";")[0].strip()
        if s.endswith(":") and " " not in s:  # labels (.LBB0_2: included) before directives
            out.append(("label", set(), set(), raw, 0, "", s[:-1]))
            continue
        if not s or s.startswith(".") or s.startswith("//"):
            out.append(("skip", set(), set(), raw, 0, "", None))
            continue
        op, _, rest = s.partition(" ")
        if op == "s_nop":
            out.append(("inst", set(), set(), raw, int(rest.strip(), 0) + 1, op, None))
            continue
        ops = [o.strip() for o in rest.split(",")] if rest else []
        dst, src = set(), set()
        if op.startswith("v_") and ops:
            if op.startswith(("v_cmp", "v_readlane", "v_readfirstlane")):
                src = regs(rest)
            else:
                dst = regs(ops[0])
                src = regs(",".join(ops[1:]))
                if "fmac" in op or "fmaak" in op or "mac_" in op:
                    src |= dst
        else:
            src = regs(rest)
        m = BRANCH.match(s)
        out.append(("inst", dst, src, raw, 1, op, m.group(2) if m else None))
    return out


def dpp_reads(raw):
    """Every VGPR a DPP instruction reads (sources, and the accumulator of v_fmac/v_mac)."""
    s = raw.split(";")[0].strip()
    op, _, rest = s.partition(" ")
    ops = [o.strip() for o in rest.split(",")]
    reads = set()
    for o in ops[1:]:
        reads |= regs(o.split(" ")[0])
    if ("fmac" in op or "mac_" in op) and ops:
        reads |= regs(ops[0])
    return reads


def _preds(ins, branches_to):
    """Control-flow predecessors of instruction index i, as a function."""
    def preds(i):
        out = []
        j = i - 1
        # labels between i and its fall-through predecessor: every branch to them is a predecessor
        while j >= 0 and ins[j][0] != "inst":
            if ins[j][0] == "label":
                out.extend(branches_to.get(ins[j][6], ()))
            j -= 1
        if j >= 0 and ins[j][5] not in NOFALL:
            out.append(j)
        return out
    return preds


def check(path, want="", verbose=True):
    lines = open(path).read().split("\n")
    bad = 0
    n_dpp = 0
    kernel = None
    body = []
    kernels = {}
    for ln in lines:
        m = re.match(r"^(_Z\S+):", ln)
        if m:
            kernel = m.group(1)
            kernels[kernel] = body = []
            continue
        if kernel is not None:
            body.append(ln)
            if "s_endpgm" in ln:
                kernel = None
    for name, body in kernels.items():
        if want not in name:
            continue
        ins = parse(body)
        branches_to = {}
        for j, t in enumerate(ins):
            if t[0] == "inst" and t[6] is not None:
                branches_to.setdefault(t[6], []).append(j)
        preds = _preds(ins, branches_to)
        for i, t in enumerate(ins):
            if t[0] != "inst" or "_dpp" not in t[3].split(";")[0]:
                continue
            n_dpp += 1
            reads = dpp_reads(t[3])
            # depth-first over predecessors while fewer than 2 wait states separate them from i
            stack = [(p, 0) for p in preds(i)]
            seen = set()
            while stack:
                j, states = stack.pop()
                if (j, states) in seen:
                    continue
                seen.add((j, states))
                _, d2, _, r2, st, _, _ = ins[j]
                if d2 & reads:
                    bad += 1
                    if verbose:
                        print(f"{name}: {r2.strip()}  ->  {t[3].strip()}  ({states} states)")
                    break
                if states + st < 2:
                    stack.extend((p, states + st) for p in preds(j))
    if verbose:
        print(f"checked {n_dpp} DPP instructions, {bad} hazards")
    return bad


if __name__ == "__main__":
    sys.exit(1 if check(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "") else 0)
