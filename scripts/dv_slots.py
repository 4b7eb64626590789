"""Experiment (measured, NOT adopted): a bank-conflict-free LDS slot map for the 12x12 symmetric
stage blocks of the register-resident solver (pdipm_srbd_reg.hpp, RegLayout::DV, which keeps the
packed lower layout r(r+1)/2 + c with stride 78). Result in profiles/r01/dv_layout_variants.txt:
LDS bank-conflict cycles -23 % per QP, but the slot lookups added VALU/LDS instructions and the
fused step measured +0.9 % (0.864 vs 0.856 ms, same box, alternating runs), so the packed layout
stays. Kept as the record of the experiment.

In the twisted block recursion lane r of each 16-lane group reads element (r, c) of its stage block
for c = 0..11, one ds_read_b64 per c, both groups in the same instruction. LDS has 64 banks of 4 B,
so a double in slot s occupies banks 2s, 2s+1 (mod 64): 32 double slots per bank cycle. With
  * slot(r, c) = slot(c, r) in 0..79, all 78 pairs distinct,
  * every column's 12 slots distinct mod 16, and
  * block stride 80 (= 16 mod 32): the two groups' blocks are 16 doubles apart mod 32 whenever their
    stages are an odd distance apart, which holds in the factorisation and the forward solve chains
    (stages t and N-1-t, N even); the back substitution (stages mid-1-t, mid+1+t) stays 2-way,
the 24 rows of one chain load land in 24 distinct bank pairs (the packed lower layout r(r+1)/2 + c
models at ~2.4 cycles per load). Placing group-0 stages at even and group-1 stages at odd block
positions would make the back substitution conflict-free too, but its index arithmetic in the
S_ii build cost more VALU than it saved (measured, profiles/r01/dv_layout_variants.txt).

python scripts/dv_slots.py  -> the table and the modelled cycles per load
"""
import collections
import random


def search(seed=1):
    pairs = [(r, c) for r in range(12) for c in range(r + 1)]
    rng = random.Random(seed)

    def cost(a):
        tot = 0
        for c in range(12):
            cnt = collections.Counter(a[(max(r, c), min(r, c))] % 16 for r in range(12))
            tot += max(cnt.values()) - 1
        return tot

    while True:
        slots = list(range(80))
        rng.shuffle(slots)
        a = dict(zip(pairs, slots[:78]))
        spare = slots[78:]
        cur = cost(a)
        for _ in range(200000):
            if cur == 0:
                return a
            p = rng.choice(pairs)
            if rng.random() < 0.2:  # move to a spare slot
                k = rng.randrange(len(spare))
                a[p], spare[k] = spare[k], a[p]
                nc = cost(a)
                if nc <= cur:
                    cur = nc
                else:
                    a[p], spare[k] = spare[k], a[p]
            else:
                q = rng.choice(pairs)
                a[p], a[q] = a[q], a[p]
                nc = cost(a)
                if nc <= cur:
                    cur = nc
                else:
                    a[p], a[q] = a[q], a[p]


def sym(r, c):
    return r * (r + 1) // 2 + c if r >= c else c * (c + 1) // 2 + r


def model_cycles(slot, stride, base0, base1):
    def cycles(addrs):
        banks = collections.defaultdict(set)
        for a in addrs:
            for d in (2 * a, 2 * a + 1):
                banks[d % 64].add(d)
        return max(len(v) for v in banks.values())
    tot = [cycles([base0 + slot(min(l, 11), c) for l in range(16)] +
                  [base1 + slot(min(l, 11), c) for l in range(16)]) for c in range(12)]
    return sum(tot) / 12


if __name__ == "__main__":
    a = search()
    table = [a[(max(r, c), min(r, c))] for r in range(12) for c in range(r + 1)]  # by sym index
    assert sorted(table) == sorted(set(table)) and max(table) < 80
    for c in range(12):
        assert len({table[sym(r, c)] % 16 for r in range(12)}) == 12
    f = lambda r, c: table[sym(r, c)]
    print("// dv_slot[sym(r, c)]")
    print("{" + ", ".join(map(str, table)) + "}")
    print("modelled cycles per chain load (1 = conflict free):")
    print("  new, blocks 80 apart, stages 0 / 9:", model_cycles(f, 80, 0, 80 * 9))
    print("  new, blocks 80 apart, stages 4 / 6 (back substitution):", model_cycles(f, 80, 80 * 4, 80 * 6))
    print("  old packed lower, stride 78 (forward pair 0/9):",
          model_cycles(lambda r, c: sym(r, c), 78, 0, 78 * 9))
