"""Device test-set evaluation (qmfx_eval_ranks, csrc/eval.hip) against the oracle.

Bar: the scores of labelled pairs are the reference's double scores bit for bit, the
per-positive counts of higher-scored items are exact, Σ score² is within 1e-12 relative,
and every metric (mse, auc, ap, p@k, r@k) equals the oracle's dense metric (P@k/R@k exactly;
the rest within 1e-12 relative: only summation order differs).  Covers fp32 and fp64
contexts, k up to 256 (several LDS column stages), item biases, exact score ties, users
without positives, non-positive labels, and a workgroup with more positives than its LDS
counters (global-atomic path).
"""
import numpy as np
import pytest

import pyoracle as po
import qmf_amd
from qmf_amd import metrics as qm

pytestmark = pytest.mark.gpu


def _case(rng, nu, ni, k, ntest, dense_user=None):
    U = rng.normal(0, 0.3, (nu, k))
    I = rng.normal(0, 0.3, (ni, k))
    I[7] = I[3]          # exact ties: identical item rows score identically
    I[11] = I[3]
    users = rng.choice(nu, ntest, replace=False)
    rowptr, items, values = [0], [], []
    for t in range(ntest):
        m = int(rng.integers(0, 12))
        if dense_user is not None and t == dense_user:
            m = min(ni, 2600)
        it = np.sort(rng.choice(ni, m, replace=False))
        if t % 5 == 0:
            it = np.union1d(it, [3, 7, 11])
        v = rng.choice([-1.0, 0.5, 1.0, 2.0, 4.0], len(it))
        if t % 7 == 3:
            v[:] = -1.0    # no positives
        items.extend(it.tolist())
        values.extend(v.tolist())
        rowptr.append(len(items))
    return U, I, users, np.array(rowptr), np.array(items, np.int64), np.array(values)


@pytest.mark.parametrize("prec,k,bias,ni,ntest,dense", [
    (64, 16, False, 500, 40, None),
    (32, 30, True, 777, 33, None),
    (64, 130, True, 300, 20, None),
    (32, 256, False, 1000, 17, None),
    (32, 64, False, 5000, 24, 2),
])
def test_eval_ranks_match_oracle(prec, k, bias, ni, ntest, dense):
    rng = np.random.default_rng(k + ni)
    nu = 200
    U, I, users, rowptr, items, values = _case(rng, nu, ni, k, ntest, dense)
    if prec == 32:  # the device stores fp32: the reference scores those same values
        U, I = U.astype(np.float32).astype(np.float64), I.astype(np.float32).astype(np.float64)
    b = rng.normal(0, 0.5, ni) if bias else None
    if bias and prec == 32:
        b = b.astype(np.float32).astype(np.float64)
    with qmf_amd.Context(k, prec) as c:
        c.set_shape(nu, ni)
        c.set_factors(0, U)
        c.set_factors(1, I)
        if bias:
            c.bpr_set_biases(b)
        c.eval_set_labels(users, rowptr, items, values)
        res = c.eval_ranks(use_biases=bias)
    ls, above, sq = res
    S = po.test_scores(U, I, users, b)
    p = 0
    ranked = qm.ranked_users(res, rowptr, values, ni)
    for t in range(ntest):
        sl = slice(rowptr[t], rowptr[t + 1])
        assert np.array_equal(ls[sl], S[t, items[sl]]), t          # bit-exact scores
        labels = np.zeros(ni)
        labels[items[sl]] = values[sl]
        sq_o, _, above_o = po.rank_stats(labels, S[t])
        assert np.array_equal(above[p:p + len(above_o)], above_o), t  # exact counts
        p += len(above_o)
        assert sq[t] == pytest.approx(sq_o, rel=1e-12)
        u = ranked[t]
        tol = dict(rel=1e-12, abs=1e-15)
        assert qm.mse(u) == pytest.approx(po.metric_mse(labels, S[t]), **tol)
        npos = len(above_o)
        assert qm.auc(u) == pytest.approx(po.metric_auc(labels, S[t]), **tol)
        if npos:
            assert qm.average_precision(u) == pytest.approx(po.metric_ap(labels, S[t]), **tol)
        for kk in (1, 5, 10, 50):
            assert qm.precision(u, kk) == po.metric_precision(labels, S[t], kk)
            if npos:
                assert qm.recall(u, kk) == po.metric_recall(labels, S[t], kk)
    assert p == len(above)


def test_eval_requires_labels():
    with qmf_amd.Context(8, 32) as c:
        c.set_shape(4, 4)
        with pytest.raises(qmf_amd.QmfxError):
            c._ev = (0, 0, 0)
            c.eval_ranks()


@pytest.mark.parametrize("batch_groups", ["1", "3"])
def test_eval_user_batches_equal_one_launch(batch_groups, monkeypatch):
    """Test users beyond one launch's grid (65535 groups of 32 users, ≈2.1M users: the
    reference's --num_test_users=0 on a C3-size set) run in batches; forcing batches of 1
    and 3 groups on 150 users (5 groups, a ragged last one) must give the same statistics
    bit for bit as a single launch."""
    rng = np.random.default_rng(9)
    nu, ni, k, ntest = 400, 900, 48, 150
    U, I, users, rowptr, items, values = _case(rng, nu, ni, k, ntest)
    out = []
    for env in (None, batch_groups):
        if env:
            monkeypatch.setenv("QMFX_EVAL_BATCH_GROUPS", env)
        with qmf_amd.Context(k, 64) as c:
            c.set_shape(nu, ni)
            c.set_factors(0, U)
            c.set_factors(1, I)
            c.eval_set_labels(users, rowptr, items, values)
            out.append(c.eval_ranks())
    for a, b in zip(*out):
        assert np.array_equal(a, b)
