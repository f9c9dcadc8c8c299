"""Parity at each BASELINE.json configuration's own shape, reduced in size so the CPU oracle
finishes in seconds: the same densities (C2/C3/C5: 50 signals per user, 500 per item), the
same k, the reference's λ = 0.05, α = 40, and the device route each config takes at full
size (whitened user rows, direct or multi-wave item rows; fp32 split-bf16 Gram at k ≥ 96).

* C2 (k=64, fp32), C3 and C5 (k=128 / 256, fp32 and fp64 — fp64 is the reference's Double and
  the headline precision): two epochs in lock-step (each half checked on its own) and three
  epochs run independently, against the oracle (WALSEngine::iterate, WALSEngine.cpp:165-218).
  fp32 within 1e-4 (north_star), fp64 1e-9.
* C4 (BPR, k=64): the exact update sequence of a serial epoch at k=64, and the Hogwild
  epoch's eval-loss trajectory against a serial reference SGD on a C4-shaped matrix.

The full-size C3 matrix is checked inside bench.py (sampled rows re-solved by the oracle
against the device's own fixed side; `parity` in the BENCH line)."""
import os

import numpy as np
import pytest

import pyoracle as po
import qmf_amd
from helpers import csr_from_triples, rel_err, synth

pytestmark = pytest.mark.gpu
LAM, ALPHA = 0.05, 40.0
NTHR = min(16, len(os.sched_getaffinity(0)))


@pytest.fixture(scope="module")
def c_shape():
    # 20 000 users x 2 000 items, 1M nnz: 50 per user, 500 per item (C2/C3/C5 densities)
    return synth(20000, 2000, 1_000_000, seed=23)


def pair(u, i, v, k, precision, seed=1):
    o = po.OracleWALS(u, i, v, k, LAM, ALPHA)
    uids, iids, (urp, ucol, uval), (irp, icol, ival) = csr_from_triples(u, i, v)
    c = qmf_amd.Context(k, precision)
    c.set_shape(len(uids), len(iids))
    c.upload_csr(0, urp, ucol, uval)
    c.upload_csr(1, irp, icol, ival)
    init = np.random.default_rng(seed).uniform(-0.01, 0.01, (len(iids), k))
    o.set_factors(1, init)
    c.set_factors(1, init)
    return o, c


@pytest.mark.parametrize("cfg,k,precision", [("C2", 64, 32), ("C3", 128, 32), ("C3", 128, 64),
                                             ("C5", 256, 32), ("C5", 256, 64)])
def test_config_shape_lockstep_halves(c_shape, cfg, k, precision):
    o, c = pair(*c_shape, k, precision)
    tol = 1e-4 if precision == 32 else 1e-9
    for h in range(4):
        side = h % 2
        lo = o.iterate(side, NTHR)
        ld = c.wals_half(side, ALPHA, LAM) / (o.nusers * o.nitems)
        assert len(c.failed_rows()) == 0, (cfg, h)  # SPD rows: no pivoted re-solve
        err = rel_err(c.factors(side), o.factors(side))
        assert err < tol, (cfg, h, err)
        assert abs(ld - lo) < tol * abs(lo), (cfg, h, ld, lo)
        c.set_factors(side, o.factors(side))


@pytest.mark.parametrize("cfg,k,precision", [("C2", 64, 32), ("C3", 128, 32), ("C5", 256, 32),
                                             ("C3", 128, 64), ("C5", 256, 64)])
def test_config_shape_three_epochs(c_shape, cfg, k, precision):
    """Independent trajectories: each half's rounding feeds the next (fp64: the device's
    Cholesky against the oracle's Bunch-Kaufman dsysv, compounding over six halves)."""
    o, c = pair(*c_shape, k, precision, seed=2)
    tol = 1e-4 if precision == 32 else 1e-9
    for ep in range(3):
        lo = [o.iterate(s, NTHR) for s in (0, 1)][1]
        ld = [c.wals_half(s, ALPHA, LAM) for s in (0, 1)][1] / (o.nusers * o.nitems)
        for side in (0, 1):
            err = rel_err(c.factors(side), o.factors(side))
            assert err < tol, (cfg, ep, side, err)
        assert abs(ld - lo) < tol * abs(lo), (cfg, ep)


M64 = (1 << 64) - 1


def test_c4_bpr_update_sequence_k64():
    """BPREngine::update (BPREngine.cpp:178-220) at C4's k=64, fp32 and fp64, through the
    device's apply kernel on a C4-shaped triplet stream (every update serial)."""
    rng = np.random.default_rng(4)
    nu, ni, k = 2000, 500, 64
    trip = np.stack([rng.integers(0, nu, 20000), rng.integers(0, ni, 20000),
                     rng.integers(0, ni, 20000)], 1)
    U0 = rng.uniform(-0.01, 0.01, (nu, k))
    I0 = rng.uniform(-0.01, 0.01, (ni, k))
    for precision, tol in ((64, 1e-12), (32, 1e-5)):
        with qmf_amd.Context(k, precision) as c:
            c.set_shape(nu, ni)
            c.set_factors(0, U0)
            c.set_factors(1, I0)
            c.bpr_apply(trip, 0.05, 1.0, 0.025, 0.0025, False)
            U, I, b = U0.copy(), I0.copy(), np.zeros(ni)
            po.bpr_update_seq(U, I, b, trip, 0.05, 1.0, 0.025, 0.0025, False)
            s = max(np.abs(U).max(), np.abs(I).max())
            assert np.max(np.abs(c.factors(0) - U)) <= tol * s
            assert np.max(np.abs(c.factors(1) - I)) <= tol * s


def test_c4_bpr_hogwild_tracks_serial_sgd():
    """C4's workload shape (50 positives per user, 3 negatives, lr 0.05 decay 0.9, no
    biases, k=64) on a reduced matrix: the device Hogwild epochs' mean eval loss tracks a
    serial reference SGD from the same init (Hogwild is non-reproducible in the reference
    too)."""
    u, i, _ = synth(4000, 1000, 200000, seed=44)
    k, lr, lam, nneg = 64, 0.05, (1.0, 0.025, 0.0025), 3
    uids, iids, (urp, ucol, _), _ = csr_from_triples(u, i, np.ones(len(u)))
    nu, ni = len(uids), len(iids)
    users = np.repeat(np.arange(nu), np.diff(urp))
    perm = np.random.default_rng(1).permutation(len(users))
    pu, pi = users[perm], ucol[perm].astype(np.int64)
    rng = np.random.default_rng(5)
    U0 = rng.uniform(-0.01, 0.01, (nu, k))
    I0 = rng.uniform(-0.01, 0.01, (ni, k))
    keys = set((pu * ni + pi).tolist())
    ev = []
    for a, p in zip(pu[:20000], pi[:20000]):
        n = int(rng.integers(0, ni))
        while int(a) * ni + n in keys:
            n = int(rng.integers(0, ni))
        ev.append((a, p, n))
    ev = np.array(ev, np.int64)
    U, I, b = U0.copy(), I0.copy(), np.zeros(ni)
    sim = []
    order = np.arange(len(pu))
    for e in range(3):
        uu, pp = np.repeat(pu[order], nneg), np.repeat(pi[order], nneg)
        nn = rng.integers(0, ni, len(uu))
        bad = np.array([x in keys for x in (uu * ni + nn).tolist()])
        while bad.any():
            nn[bad] = rng.integers(0, ni, int(bad.sum()))
            bad[bad] = [x in keys for x in (uu[bad] * ni + nn[bad]).tolist()]
        po.bpr_update_seq(U, I, b, np.stack([uu, pp, nn], 1), lr * 0.9 ** e, *lam, False)
        sim.append(po.bpr_loss_sum(U, I, b, ev, False) / len(ev))
        order = rng.permutation(order)
    with qmf_amd.Context(k, 32) as c:
        c.set_shape(nu, ni)
        c.bpr_set_positives(pu, pi)
        c.set_factors(0, U0)
        c.set_factors(1, I0)
        dev = []
        for e in range(3):
            c.bpr_epoch(100 + e, nneg, lr * 0.9 ** e, *lam, False, shuffle=e > 0)
            dev.append(c.bpr_eval(0, ev, False) / len(ev))
    assert dev[-1] < dev[0] < np.log(2.0)
    for e in range(3):
        assert abs(dev[e] - sim[e]) < 0.01, (e, dev, sim)
