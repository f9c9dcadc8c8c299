"""Phase split of the k > 128 fp64 row kernel's LDLᵀ factorization (diagnostics): run one
C5-shaped item half with QMFX_TRACE on a library built with -DQMFX_BIG_SUBTRACE
(tools/build_variant.sh, SRC=wals_big) and print the median cycles per 500-signal row of the
Gram, the panel stores (a), the panel factorization (b), the trailing update (c) (each with
the barrier behind it) and the backward solve.
usage: QMFX_LIB=qmf_amd/_build/var_sub.so python tools/big_subtrace.py [nu ni nnz k]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
path = os.path.join(ROOT, "gpurun_out", "subtrace")
os.environ["QMFX_TRACE"] = path
import qmf_amd  # noqa: E402

cfg = [int(x) for x in sys.argv[1:5]] if len(sys.argv) > 4 else [10_000_000, 1_000_000, 500_000_000, 256]
c = qmf_amd.Context(cfg[3], 64)
c.gen_synthetic(cfg[0], cfg[1], cfg[2], 3)
c.fill_uniform(1, 0.01, 103)
c.fill_uniform(0, 0.01, 104)
for _ in range(2):
    c.wals_half(1, 40.0, 0.05)
t = np.fromfile(path + "_side1.bin", dtype=np.uint64).reshape(-1, 8).astype(np.int64)
os.remove(path + "_side1.bin")
t = t[t[:, 0] > 0]
n = t[:, 6]
m = (n >= 401) & (n <= 600)
med = np.median(t[m][:, [5, 1, 2, 3, 4]], axis=0)
print("rows %d (n 401-600 of %d traced)" % (m.sum(), len(t)))
for name, v in zip(["Gram", "(a) panel stores", "(b) panel factor", "(c) trailing", "backward"], med):
    print("%-18s %8.0f cycles" % (name, v))
print("factorization + backward %8.0f" % med[1:].sum())
