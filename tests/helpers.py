"""Shared helpers for the parity tests (fixture loading, reference-format text)."""
import hashlib
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def load_ml100k():
    z = np.load(os.path.join(GOLDEN, "ml100k_shape.npz"))
    d = {k: z[k] for k in z.files}
    d["users"] = d["users"].astype(np.int64)
    d["items"] = d["items"].astype(np.int64)
    d["values"] = d["values"].astype(np.float64)
    d["init"] = d["init_e9"].astype(np.float64) / 1e9
    return d


def load_tiny():
    a = np.loadtxt(os.path.join(GOLDEN, "tiny.txt"), dtype=np.int64)
    return a[:, 0], a[:, 1], a[:, 2].astype(np.float64)


def factor_text(ids, F):
    """Engine::saveFactors format (Engine.cpp:98-122): id then ' %.9f' per factor."""
    return "".join(str(int(i)) + "".join(" %.9f" % x for x in row) + "\n" for i, row in zip(ids, F))


def md5(s):
    return hashlib.md5(s.encode()).hexdigest()


def synth(nusers, nitems, nnz, seed, wmax=5):
    """Uniform unique (u, i) pairs with w in 1..wmax, shuffled (SURVEY.md §8(d) recipe)."""
    rng = np.random.default_rng(seed)
    keys = np.unique(rng.integers(0, nusers * nitems, size=int(nnz * 1.2)))
    keys = rng.permutation(keys)[:nnz]
    return (keys // nitems).astype(np.int64), (keys % nitems).astype(np.int64), \
        rng.integers(1, wmax + 1, size=len(keys)).astype(np.float64)


def rel_err(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


def csr_from_triples(users, items, values):
    """Independent numpy restatement of groupSignals (WALSEngine.cpp:130-163): ids sorted
    ascending as signed int64 give idx 0..n-1; each row's signals sorted by the other id;
    duplicates kept.  Returns (uids, iids, (urp, ucol, uval), (irp, icol, ival))."""
    users = np.asarray(users, np.int64)
    items = np.asarray(items, np.int64)
    values = np.asarray(values, np.float64)
    uids, uidx = np.unique(users, return_inverse=True)
    iids, iidx = np.unique(items, return_inverse=True)

    def side(rows, cols, nrows):
        order = np.lexsort((cols, rows))  # stable: by row, then col
        rp = np.zeros(nrows + 1, np.int64)
        np.add.at(rp, rows + 1, 1)
        return np.cumsum(rp), cols[order].astype(np.int32), values[order]

    return uids, iids, side(uidx, iidx, len(uids)), side(iidx, uidx, len(iids))
