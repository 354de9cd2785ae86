#!/usr/bin/env python3
"""Search for a conflict-free(er) row schedule under the LDS bank model of
scripts/lds_bank_model.py: permute each row's edges across the dc gather/scatter
instructions and move rows between thread slots (both invisible to the results:
the fast check node is order-free). Prints the modelled LDS cycles per
codeword-iteration before and after. Exploration tool for the host-side
schedule optimiser in graph.cpp."""
import sys
import numpy as np

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from lds_bank_model import load, read_b64, write_b64, model  # noqa: E402


def main():
    s = load(sys.argv[1])
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
    rng = np.random.default_rng(1)
    N, T, rpt, dc, e_pad = s["N"], s["T"], s["rpt"], s["dc"], s["e_pad"]
    R = T * rpt
    cols = s["cols"].copy()
    pos = s["pos"].copy()
    cols[s["deg"] == 0] = N + 2
    c2v_base = 8 * (N + 3)
    # slot index of row-slot q: wave w = (q % T) // 64, r = q // T, lane = q % 64
    def instr_rows(w, r):
        return np.arange(64) + 64 * w + r * T

    def cost_wr_k(w, r, k):
        rows = instr_rows(w, r)
        return read_b64(8 * cols[rows, k]) + write_b64(c2v_base + 8 * pos[rows, k])

    def cost_all():
        return sum(cost_wr_k(w, r, k) for w in range(T // 64) for r in range(rpt) for k in range(dc))

    base = cost_all()
    print("gather+scatter modelled", base, "conflict-free", (T // 64) * rpt * dc * 8)
    cur = base
    wr_of = lambda q: ((q % T) // 64, q // T)
    for it in range(iters):
        if rng.random() < 0.7:
            q = int(rng.integers(R))
            k1, k2 = rng.choice(dc, 2, replace=False)
            w, r = wr_of(q)
            before = cost_wr_k(w, r, k1) + cost_wr_k(w, r, k2)
            cols[q, [k1, k2]] = cols[q, [k2, k1]]
            pos[q, [k1, k2]] = pos[q, [k2, k1]]
            after = cost_wr_k(w, r, k1) + cost_wr_k(w, r, k2)
            if after > before:
                cols[q, [k1, k2]] = cols[q, [k2, k1]]
                pos[q, [k1, k2]] = pos[q, [k2, k1]]
            else:
                cur += after - before
        else:
            q1, q2 = (int(x) for x in rng.choice(R, 2, replace=False))
            (w1, r1), (w2, r2) = wr_of(q1), wr_of(q2)
            if (w1, r1) == (w2, r2):
                continue
            before = sum(cost_wr_k(w1, r1, k) + cost_wr_k(w2, r2, k) for k in range(dc))

            def swap():
                cols[[q1, q2]] = cols[[q2, q1]]
                p1, p2 = pos[q1].copy(), pos[q2].copy()
                # padding edges write the lane's own dummy slot
                l1, l2 = q1 % 64, q2 % 64
                p1 = np.where(p1 >= e_pad, e_pad + l2, p1)
                p2 = np.where(p2 >= e_pad, e_pad + l1, p2)
                pos[q1], pos[q2] = p2, p1
            swap()
            after = sum(cost_wr_k(w1, r1, k) + cost_wr_k(w2, r2, k) for k in range(dc))
            if after > before:
                swap()
            else:
                cur += after - before
        if it % 5000 == 0:
            print(it, cur, flush=True)
    print("final", cur, "check", cost_all())


if __name__ == "__main__":
    main()
