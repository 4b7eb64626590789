"""Static check of the VALU-write -> DPP-read hazard (2 wait states) in a kernel's ISA, inline asm
included: for every DPP instruction, the instructions issued in the 2 wait states before it must not
write a VGPR it reads. s_nop N counts N + 1 states, other instructions 1; the scan follows the
straight-line predecessor and stops at a label (a branch target's other predecessors are not
followed). Used to audit the asm blocks' wait states (csrc/pdipm_srbd.hpp SRBD_ASM_TAIL).

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -DSRBD_SPLIT_REG20 --cuda-device-only -S \
        -o /tmp/k.s biped_pympc_amd/csrc/srbd_mpc.hip
    python scripts/dpp_hazard_check.py /tmp/k.s [kernel-symbol-substring]
"""
import re
import sys

REG = re.compile(r"\bv(\d+)\b|\bv\[(\d+):(\d+)\]")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(1) is not None:
            out.add(int(m.group(1)))
        else:
            out.update(range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def parse(lines):
    """(kind, dst_regs, src_regs, text, states) per line; kind: 'label', 'inst', 'skip'."""
    out = []
    for raw in lines:
        s = raw.split(";")[0].strip()
        if not s or s.startswith(".") or s.startswith("//"):
            out.append(("skip", set(), set(), raw, 0))
            continue
        if s.endswith(":"):
            out.append(("label", set(), set(), raw, 0))
            continue
        op, _, rest = s.partition(" ")
        if op == "s_nop":
            out.append(("inst", set(), set(), raw, int(rest.strip(), 0) + 1))
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
        out.append(("inst", dst, src, raw, 1))
    return out


def check(path, want=""):
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
        for i, (kind, dst, src, raw, _) in enumerate(ins):
            if kind != "inst" or "_dpp" not in raw.split(";")[0]:
                continue
            n_dpp += 1
            s = raw.split(";")[0].strip()
            op, _, rest = s.partition(" ")
            ops = [o.strip() for o in rest.split(",")]
            # the DPP-routed operand, src0 (the second operand of v_*_dpp D, S0, ...). The blocks'
            # accumulator chains read their FMAC accumulator (src2 = D) 1-2 states after writing it,
            # as they have since round 1 with results at the oracle's FP64 floor: the hardware
            # hazard is on the routed operand (LLVM's recognizer checks every VGPR use)
            reads = regs(ops[1]) if len(ops) > 1 else set()
            states = 0
            j = i - 1
            while j >= 0 and states < 2:
                k2, d2, _, r2, st = ins[j]
                if k2 == "label":
                    break
                if k2 == "inst":
                    if d2 & reads:
                        bad += 1
                        print(f"{name}: {r2.strip()}  ->  {raw.strip()}  ({states} states)")
                        break
                    states += st
                j -= 1
    print(f"checked {n_dpp} DPP instructions, {bad} hazards")
    return bad


if __name__ == "__main__":
    sys.exit(1 if check(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "") else 0)
