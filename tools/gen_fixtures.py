"""Generates the committed golden fixtures under tests/golden/.

* ml100k_shape.npz — SURVEY.md Appendix C's ML-100K-shaped synthetic (943 users × 1682
  items, 100 000 unique pairs, w ∈ 1..5, numpy default_rng(1234)) plus its
  `--distribution_file` init (U(−0.01, 0.01), 1682·128 values written "%.9f", so the stored
  values are the %.9f-rounded ones the reference reads back).  Expected outputs recorded
  with it come from the REFERENCE itself as measured by the survey: epoch-1 loss 1.81858,
  epoch-10 loss 0.574536 (k=30, λ=0.05, α=40, OMP_NUM_THREADS=1) and the md5 prefixes of
  the saved factor files (U 7bca0507…, I 7d0e032b…).  The full md5s below were produced by
  the oracle routed through MKL's dsysv_ and agree with those prefixes.
* tiny.txt — a small "u i w" file with the bookkeeping edge cases of SURVEY.md §0.6:
  duplicate (u, i) pairs, zero values, negative and non-contiguous int64 ids, a user with a
  single interaction.

Run: python tools/gen_fixtures.py   (numpy 2.2.6; deterministic)
"""
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "..", "tests", "golden")

NU, NI, NNZ = 943, 1682, 100000


def ml100k_shape():
    rng = np.random.default_rng(1234)
    seen = {}
    while len(seen) < NNZ:  # draw pairs in batches until 100 000 unique ones
        u = rng.integers(1, NU + 1, size=NNZ)
        i = rng.integers(1, NI + 1, size=NNZ)
        for a, b in zip(u.tolist(), i.tolist()):
            if (a, b) not in seen:
                seen[(a, b)] = 1
                if len(seen) == NNZ:
                    break
    pairs = np.array(sorted(seen), np.int64)
    pairs = pairs[rng.permutation(len(pairs))]
    w = rng.integers(1, 6, size=len(pairs))
    init = rng.uniform(-0.01, 0.01, NI * 128)
    init_e9 = np.array([int(round(float("%.9f" % x) * 1e9)) for x in init], np.int32)
    return pairs[:, 0].astype(np.int16), pairs[:, 1].astype(np.int16), w.astype(np.int8), init_e9


def tiny():
    rng = np.random.default_rng(7)
    users = np.array([-5, 3, 17, 1 << 40, -(1 << 33), 99, 1000003, 42, 8, 2], np.int64)
    items = np.array([11, -2, 7, 1 << 35, 500, 6, -(1 << 50), 13, 21, 4, 999, 3], np.int64)
    lines = []
    for u in users[1:]:
        for i in rng.choice(items, size=rng.integers(3, 9), replace=False):
            lines.append((int(u), int(i), int(rng.integers(0, 6))))
    lines.append((int(users[0]), int(items[2]), 4))  # user with one interaction
    lines.append((lines[3][0], lines[3][1], 2))  # duplicate pair, kept twice
    lines.append((lines[5][0], lines[5][1], 0))  # duplicate with a zero value
    order = rng.permutation(len(lines))
    return [lines[j] for j in order]


def main():
    os.makedirs(GOLDEN, exist_ok=True)
    u, i, w, init_e9 = ml100k_shape()
    np.savez_compressed(
        os.path.join(GOLDEN, "ml100k_shape.npz"), users=u, items=i, values=w, init_e9=init_e9,
        ref_loss_epoch1=np.float64(1.81858), ref_loss_epoch10=np.float64(0.574536),
        ref_md5_user="7bca0507ff502106c4b0cbdf940bb680",
        ref_md5_item="7d0e032b43ed6fc7b23e8d8bf69d88b2")
    with open(os.path.join(GOLDEN, "tiny.txt"), "w") as f:
        for a, b, c in tiny():
            f.write("%d %d %d\n" % (a, b, c))


if __name__ == "__main__":
    main()
