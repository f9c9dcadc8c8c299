"""Experiment: one device BPR epoch (qmfx_bpr_epoch, Hogwild) vs the same hyper-parameters
applied serially on the device (qmfx_bpr_apply with host-sampled triplets) vs the oracle."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import pyoracle as po  # noqa: E402
import qmf_amd  # noqa: E402
from test_cli_gpu import clustered  # noqa: E402

u, i, v = clustered(2000, 500, 30000, seed=8)
uids, iids, ev, tev = po.bpr_sets(u, i, v)
um = {x: n for n, x in enumerate(uids.tolist())}
im = {x: n for n, x in enumerate(iids.tolist())}
U_idx = np.array([um[x] for x in u.tolist()])
I_idx = np.array([im[x] for x in i.tolist()])
nu, ni, k = len(uids), len(iids), 16
rng = np.random.default_rng(0)
U0 = rng.uniform(-0.1, 0.1, (nu, k))
I0 = rng.uniform(-0.1, 0.1, (ni, k))
b0 = rng.uniform(-0.1, 0.1, ni)
lam = (1.0, 0.025, 0.0025)


def ctx():
    c = qmf_amd.Context(k, 64)
    c.set_shape(nu, ni)
    c.bpr_set_positives(U_idx, I_idx)
    c.set_factors(0, U0)
    c.set_factors(1, I0)
    c.bpr_set_biases(b0)
    return c


def loss(c):
    return c.bpr_eval(0, ev, True) / len(ev)


pos = set((U_idx * ni + I_idx).tolist())
uu = np.repeat(U_idx, 3)
pp = np.repeat(I_idx, 3)
nn = rng.integers(0, ni, len(uu))
bad = np.array([x in pos for x in (uu * ni + nn).tolist()])
while bad.any():
    nn[bad] = rng.integers(0, ni, int(bad.sum()))
    bad[bad] = [x in pos for x in (uu[bad] * ni + nn[bad]).tolist()]
trip = np.stack([uu, pp, nn], 1)

c1 = ctx()
print("init loss", loss(c1))
c1.bpr_epoch(123, 3, 0.1, *lam, True, shuffle=False)
print("device epoch (hogwild)", loss(c1))
c2 = ctx()
c2.bpr_apply(trip, 0.1, *lam, True)
print("device apply (serial)", loss(c2))
U, I, b = U0.copy(), I0.copy(), b0.copy()
po.bpr_update_seq(U, I, b, trip, 0.1, *lam, True)
print("oracle serial", po.bpr_loss_sum(U, I, b, ev, True) / len(ev))
print("apply vs oracle max diff", np.abs(c2.factors(0) - U).max(), np.abs(c2.factors(1) - I).max())
for w in range(3):
    c1.bpr_epoch(1000 + w, 3, 0.1 * 0.9 ** (w + 1), *lam, True, shuffle=True)
    print("device epoch", w + 2, loss(c1))
