"""Entry order of the S_ii build (csrc/srbd_common.hpp kSiiOrder, the TRI table of
pdipm_srbd_reg.hpp factor_build): which lane computes which packed entry (r, c) of the 12x12
stage block. Each lane writes its entry with ds_write_b64 to slot kDvSlot[(r, c)] of the stage's
block; a ds_write_b64 serves 16 contiguous lanes per LDS cycle with bank (address / 4) mod 32, i.e.
slot mod 16, so lanes of one 16-group writing slots with equal residues conflict. The kDvSlot map is
fixed by the block chains (conflict-free column reads), so only the order within the two classes is
free: dense x dense (21 entries; lanes 21 q + k write stage blocks q = 0, 1, 2 at once, 80 doubles
= 0 mod 16 apart) and the 57 entries with a sparse index (one stage block per trip). A seeded local
search minimises the extra write cycles: dense 6 -> 5, sparse 4 -> 2 per write instruction, i.e.
64 -> 40 bank-conflict cycles per Newton iteration and QP at N = 10 (4 dense + 10 sparse writes).

    python scripts/sii_order.py        (prints the C++ table)
"""
import random
from collections import Counter

K_DV_SLOT = [77, 58, 32, 73, 46, 5, 52, 54, 50, 65, 53, 75, 31, 14, 76, 30, 69, 71, 64, 20, 15, 48, 8, 3, 9, 23,
             28, 21, 6, 49, 43, 44, 29, 18, 78, 51, 19, 61, 42, 79, 41, 24, 33, 39, 70, 55, 2, 22, 37, 40, 67, 27,
             26, 68, 60, 66, 57, 36, 59, 1, 45, 74, 56, 0, 63, 7, 11, 12, 72, 10, 35, 25, 4, 16, 34, 62, 38, 13]


def sym(r, c):
    return r * (r + 1) // 2 + c if r >= c else c * (c + 1) // 2 + r


def class_entries():
    out = []
    for cls in range(3):
        for r in range(12):
            for c in range(r + 1):
                if (r % 6 >= 3) + (c % 6 >= 3) == cls:
                    out.append((r, c))
    return out[:21], out[21:]


def write_conflicts(lane_entry):
    """Extra LDS cycles of one ds_write_b64 by lanes -> entries (4 groups of 16 contiguous lanes)."""
    tot = 0
    for g in range(4):
        res = Counter(K_DV_SLOT[sym(*lane_entry[l])] % 16 for l in range(16 * g, 16 * g + 16) if l in lane_entry)
        tot += max(res.values()) - 1 if res else 0
    return tot


def dense_cost(order):
    return write_conflicts({lw: order[lw % 21] for lw in range(63)})


def sparse_cost(order):
    return write_conflicts({lw: order[lw] for lw in range(57)})


def search(order, cost, iters=200000, seed=1):
    rng = random.Random(seed)
    best, bo = cost(order), list(order)
    for _ in range(iters):
        o = list(bo)
        i, j = rng.sample(range(len(o)), 2)
        o[i], o[j] = o[j], o[i]
        v = cost(o)
        if v <= best:
            best, bo = v, o
    return bo, best


if __name__ == "__main__":
    d0, s0 = class_entries()
    dn, dc = search(d0, dense_cost)
    sn, sc = search(s0, sparse_cost)
    print(f"// dense {dense_cost(d0)} -> {dc}, sparse {sparse_cost(s0)} -> {sc} extra cycles per write")
    print("constexpr uint8_t kSiiOrder[78] = {" + ", ".join(str(r | (c << 4)) for r, c in dn + sn) + "};")
