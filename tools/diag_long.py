"""Diagnostic: fp32 direct-path error vs the oracle for long rows, by k and row length."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402
from helpers import synth, rel_err  # noqa: E402
from test_wals_gpu import make_pair  # noqa: E402

ALPHA_ = float(os.environ.get("ALPHA", "40"))
for k, prec in ((64, 32), (96, 32), (128, 32), (96, 64)):
    for nitems in (60, 300):
        u, i, v = synth(12000, nitems, 30000, seed=k)
        o, c = make_pair(u, i, v, k, prec, seed=4, lam=5.0, alpha=ALPHA_)
        o.iterate(0)
        c.wals_half(0, ALPHA_, 5.0)
        e0 = rel_err(c.factors(0), o.factors(0))
        c.set_factors(0, o.factors(0))
        o.iterate(1)
        c.wals_half(1, ALPHA_, 5.0)
        e1 = rel_err(c.factors(1), o.factors(1))
        F, R = c.factors(1), o.factors(1)
        row = int(np.argmax(np.max(np.abs(F - R), axis=1)))
        print(f"k={k} prec={prec} nitems={nitems} avg_row={30000 / nitems:.0f} "
              f"err_users={e0:.2e} err_items={e1:.2e} worst_item={row}", flush=True)
