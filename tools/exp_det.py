"""Loss determinism check: the same half on identical contexts, 1 piece vs 1 piece vs 7."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import qmf_amd  # noqa: E402
from helpers import csr_from_triples, synth  # noqa: E402

u, i, v = synth(3000, 700, 60000, seed=5)
uids, iids, (urp, ucol, uval), (irp, icol, ival) = csr_from_triples(u, i, v)
init = np.random.default_rng(4).uniform(-0.01, 0.01, (len(iids), 64))


def ctx(pieces):
    os.environ["QMFX_PIECES"] = str(pieces)
    c = qmf_amd.Context(64, 32)
    c.set_shape(len(uids), len(iids))
    c.upload_csr(0, urp, ucol, uval)
    c.upload_csr(1, irp, icol, ival)
    c.set_factors(1, init)
    return c


ref = None
n = np.diff(urp)
for p in (1, 7, 3):
    c = ctx(p)
    c.wals_half(0, 40.0, 0.05)
    rl = c.row_losses(0)
    if ref is None:
        ref = rl
        continue
    d = np.nonzero(rl != ref)[0]
    print(p, "rows differing:", len(d), "signal counts:", np.bincount(n[d])[:80].nonzero()[0][:40],
          "max rel", float(np.max(np.abs(rl[d] - ref[d]) / np.abs(ref[d]))) if len(d) else 0)
