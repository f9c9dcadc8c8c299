"""ctypes front-end for the CPU oracle (oracle/qmf_oracle.cpp).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg.  The product path (qmf_amd/) never imports this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None

c_i64p = ctypes.POINTER(ctypes.c_int64)
c_i32p = ctypes.POINTER(ctypes.c_int32)
c_f64p = ctypes.POINTER(ctypes.c_double)


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        vp = ctypes.c_void_p
        L.orc_wals_create.restype = vp
        L.orc_wals_create.argtypes = [c_i64p, c_i64p, c_f64p, ctypes.c_int64, ctypes.c_int,
                                      ctypes.c_double, ctypes.c_double]
        L.orc_wals_create_csr.restype = vp
        L.orc_wals_create_csr.argtypes = [ctypes.c_int64, ctypes.c_int64, c_i64p, c_i32p, c_f64p,
                                          c_i64p, c_i32p, c_f64p, ctypes.c_int,
                                          ctypes.c_double, ctypes.c_double]
        L.orc_wals_destroy.argtypes = [vp]
        for f in ("orc_wals_nusers", "orc_wals_nitems", "orc_wals_nnz"):
            getattr(L, f).restype = ctypes.c_int64
            getattr(L, f).argtypes = [vp]
        L.orc_wals_ids.argtypes = [vp, ctypes.c_int, c_i64p]
        L.orc_wals_csr.argtypes = [vp, ctypes.c_int, c_i64p, c_i64p, c_f64p]
        L.orc_wals_set_factors.argtypes = [vp, ctypes.c_int, c_f64p]
        L.orc_wals_get_factors.argtypes = [vp, ctypes.c_int, c_f64p]
        L.orc_wals_load_distribution_file.restype = ctypes.c_int64
        L.orc_wals_load_distribution_file.argtypes = [vp, ctypes.c_int, ctypes.c_char_p]
        L.orc_wals_iterate.restype = ctypes.c_double
        L.orc_wals_iterate.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
        L.orc_wals_optimize.argtypes = [vp, ctypes.c_int, ctypes.c_int, c_f64p]
        L.orc_wals_time_sample.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int64,
                                           c_f64p, c_f64p, c_i64p]
        L.orc_xtx.argtypes = [c_f64p, ctypes.c_int64, ctypes.c_int, c_f64p]
        L.orc_linear_symmetric_solve.restype = ctypes.c_int
        L.orc_linear_symmetric_solve.argtypes = [c_f64p, c_f64p, ctypes.c_int]
        L.orc_solve_rows.restype = ctypes.c_int
        L.orc_solve_rows.argtypes = [c_f64p, ctypes.c_int64, ctypes.c_int, c_i64p, c_i32p, c_f64p,
                                     c_i64p, ctypes.c_int64, ctypes.c_double, ctypes.c_double,
                                     ctypes.c_int, c_f64p, c_f64p]
        L.orc_update_one.restype = ctypes.c_double
        L.orc_update_one.argtypes = [c_f64p, ctypes.c_int64, ctypes.c_int, c_i64p, c_f64p,
                                     ctypes.c_int64, c_f64p, ctypes.c_double, ctypes.c_double,
                                     c_f64p]
        L.orc_bpr_predict_difference.restype = ctypes.c_double
        L.orc_bpr_predict_difference.argtypes = [c_f64p, c_f64p, c_f64p, ctypes.c_int,
                                                 ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                                 ctypes.c_int]
        L.orc_bpr_update_seq.restype = ctypes.c_int
        L.orc_bpr_update_seq.argtypes = [c_f64p, c_f64p, c_f64p, ctypes.c_int, c_i64p,
                                         ctypes.c_int64, ctypes.c_double, ctypes.c_double,
                                         ctypes.c_double, ctypes.c_double, ctypes.c_int]
        L.orc_bpr_loss_sum.restype = ctypes.c_double
        L.orc_bpr_loss_sum.argtypes = [c_f64p, c_f64p, c_f64p, ctypes.c_int, c_i64p,
                                       ctypes.c_int64, ctypes.c_int]
        L.orc_bpr_hogwild_epoch.restype = ctypes.c_int
        L.orc_bpr_hogwild_epoch.argtypes = [c_f64p, c_f64p, c_f64p, ctypes.c_int, c_i64p, c_i64p,
                                            ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                            ctypes.c_int, ctypes.c_int, ctypes.c_uint64,
                                            ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                            ctypes.c_double, ctypes.c_int, c_i64p, ctypes.c_int64,
                                            c_f64p, c_f64p, c_f64p]
        L.orc_bpr_sets.restype = ctypes.c_int
        L.orc_bpr_sets.argtypes = [c_i64p, c_i64p, c_f64p, ctypes.c_int64, c_i64p, c_i64p,
                                   c_f64p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32,
                                   c_i64p, c_i64p, c_i64p, c_i64p, c_i64p, c_i64p, c_i64p,
                                   c_i64p]
        _lib = L
    return _lib


def _p(a, t):
    if not a.flags.c_contiguous:
        raise ValueError("oracle arrays must be C-contiguous")
    return a.ctypes.data_as(t)


class OracleWALS:
    """WALSEngine restatement (WALSEngine.cpp:37-355) on one dataset."""

    def __init__(self, users, items, values, nfactors, lam=0.05, alpha=40.0):
        L = lib()
        u = np.ascontiguousarray(users, dtype=np.int64)
        i = np.ascontiguousarray(items, dtype=np.int64)
        v = np.ascontiguousarray(values, dtype=np.float64)
        self.k = int(nfactors)
        self.h = L.orc_wals_create(_p(u, c_i64p), _p(i, c_i64p), _p(v, c_f64p), len(u), self.k,
                                   float(lam), float(alpha))

    @classmethod
    def from_csr(cls, nusers, nitems, urp, ucol, uval, irp, icol, ival, nfactors, lam, alpha):
        self = cls.__new__(cls)
        L = lib()
        self.k = int(nfactors)
        arrs = [np.ascontiguousarray(urp, np.int64), np.ascontiguousarray(ucol, np.int32),
                np.ascontiguousarray(uval, np.float64), np.ascontiguousarray(irp, np.int64),
                np.ascontiguousarray(icol, np.int32), np.ascontiguousarray(ival, np.float64)]
        self._keep = arrs
        self.h = L.orc_wals_create_csr(nusers, nitems, _p(arrs[0], c_i64p), _p(arrs[1], c_i32p),
                                       _p(arrs[2], c_f64p), _p(arrs[3], c_i64p),
                                       _p(arrs[4], c_i32p), _p(arrs[5], c_f64p), self.k,
                                       float(lam), float(alpha))
        return self

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_wals_destroy(self.h)
            self.h = None

    @property
    def nusers(self):
        return lib().orc_wals_nusers(self.h)

    @property
    def nitems(self):
        return lib().orc_wals_nitems(self.h)

    @property
    def nnz(self):
        return lib().orc_wals_nnz(self.h)

    def ids(self, side):
        n = self.nusers if side == 0 else self.nitems
        out = np.empty(n, np.int64)
        lib().orc_wals_ids(self.h, side, _p(out, c_i64p))
        return out

    def csr(self, side):
        n = self.nusers if side == 0 else self.nitems
        rp = np.empty(n + 1, np.int64)
        col = np.empty(self.nnz, np.int64)
        val = np.empty(self.nnz, np.float64)
        lib().orc_wals_csr(self.h, side, _p(rp, c_i64p), _p(col, c_i64p), _p(val, c_f64p))
        return rp, col, val

    def set_factors(self, side, f):
        f = np.ascontiguousarray(f, np.float64)
        n = self.nusers if side == 0 else self.nitems
        assert f.shape == (n, self.k)
        lib().orc_wals_set_factors(self.h, side, _p(f, c_f64p))

    def factors(self, side):
        n = self.nusers if side == 0 else self.nitems
        out = np.empty((n, self.k), np.float64)
        lib().orc_wals_get_factors(self.h, side, _p(out, c_f64p))
        return out

    def load_distribution_file(self, path, side=1):
        return lib().orc_wals_load_distribution_file(self.h, side, path.encode())

    def iterate(self, side, nthreads=1):
        info = ctypes.c_int(0)
        loss = lib().orc_wals_iterate(self.h, side, nthreads, ctypes.byref(info))
        if info.value != 0:
            raise RuntimeError("dsysv failed, info=%d" % info.value)
        return loss

    def optimize(self, nepochs, nthreads=1):
        out = np.empty(nepochs, np.float64)
        lib().orc_wals_optimize(self.h, nepochs, nthreads, _p(out, c_f64p))
        return out

    def time_sample(self, side, nthreads, stride):
        a = np.zeros(2, np.float64)
        n = np.zeros(1, np.int64)
        lib().orc_wals_time_sample(self.h, side, nthreads, int(stride), _p(a[:1], c_f64p),
                                   _p(a[1:], c_f64p), _p(n, c_i64p))
        return float(a[0]), float(a[1]), int(n[0])


def xtx(X):
    X = np.ascontiguousarray(X, np.float64)
    out = np.empty((X.shape[1], X.shape[1]), np.float64)
    lib().orc_xtx(_p(X, c_f64p), X.shape[0], X.shape[1], _p(out, c_f64p))
    return out


def linear_symmetric_solve(A, b):
    A = np.ascontiguousarray(A, np.float64)
    x = np.array(b, np.float64)
    info = lib().orc_linear_symmetric_solve(_p(A, c_f64p), _p(x, c_f64p), A.shape[0])
    if info != 0:
        raise RuntimeError("dsysv info=%d" % info)
    return x


def update_one(Y, cols, vals, YtY, alpha, lam):
    Y = np.ascontiguousarray(Y, np.float64)
    cols = np.ascontiguousarray(cols, np.int64)
    vals = np.ascontiguousarray(vals, np.float64)
    YtY = np.ascontiguousarray(YtY, np.float64)
    k = Y.shape[1]
    x = np.empty(k, np.float64)
    loss = lib().orc_update_one(_p(Y, c_f64p), Y.shape[0], k, _p(cols, c_i64p), _p(vals, c_f64p),
                                len(cols), _p(YtY, c_f64p), float(alpha), float(lam),
                                _p(x, c_f64p))
    return x, loss


def solve_rows(Y, rowptr, col, val, rows, alpha, lam, nthreads=1):
    """updateFactorsForOne (WALSEngine.cpp:266-310) for the given rows of a CSR whose column
    indices index Y directly; YtY over all of Y.  Returns (x [len(rows)×k], row losses)."""
    Y = np.ascontiguousarray(Y, np.float64)
    rowptr = np.ascontiguousarray(rowptr, np.int64)
    col = np.ascontiguousarray(col, np.int32)
    val = np.ascontiguousarray(val, np.float64)
    rows = np.ascontiguousarray(rows, np.int64)
    k = Y.shape[1]
    x = np.empty((len(rows), k), np.float64)
    loss = np.empty(len(rows), np.float64)
    info = lib().orc_solve_rows(_p(Y, c_f64p), Y.shape[0], k, _p(rowptr, c_i64p), _p(col, c_i32p),
                                _p(val, c_f64p), _p(rows, c_i64p), len(rows), float(alpha),
                                float(lam), int(nthreads), _p(x, c_f64p), _p(loss, c_f64p))
    if info != 0:
        raise RuntimeError("dsysv info=%d" % info)
    return x, loss


def bpr_update_seq(U, I, bias, triplets, lr, bias_lambda, user_lambda, item_lambda, use_biases):
    """In-place BPREngine::update over triplets (BPREngine.cpp:178-220)."""
    for a in (U, I, bias):
        assert a.dtype == np.float64 and a.flags.c_contiguous, "in-place arrays must be C-contiguous f64"
    k = U.shape[1]
    t = np.ascontiguousarray(triplets, np.int64)
    rc = lib().orc_bpr_update_seq(_p(U, c_f64p), _p(I, c_f64p), _p(bias, c_f64p), k,
                                  _p(t, c_i64p), len(t), lr, bias_lambda, user_lambda,
                                  item_lambda, int(use_biases))
    if rc:
        raise FloatingPointError("gradients too big")


def bpr_predict_difference(U, I, bias, u, p, n, use_biases):
    U, I, bias = (np.ascontiguousarray(a, np.float64) for a in (U, I, bias))
    return lib().orc_bpr_predict_difference(_p(U, c_f64p), _p(I, c_f64p), _p(bias, c_f64p),
                                            U.shape[1], u, p, n, int(use_biases))


def bpr_loss_sum(U, I, bias, triplets, use_biases):
    U, I, bias = (np.ascontiguousarray(a, np.float64) for a in (U, I, bias))
    t = np.ascontiguousarray(triplets, np.int64)
    return lib().orc_bpr_loss_sum(_p(U, c_f64p), _p(I, c_f64p), _p(bias, c_f64p), U.shape[1],
                                  _p(t, c_i64p), len(t), int(use_biases))


def bpr_hogwild_epoch(U, I, bias, pos_user, pos_item, nitems, num_neg, nthreads, seed, lr,
                      bias_lambda, user_lambda, item_lambda, use_biases, eval_set):
    """One reference-structure Hogwild BPR epoch + evaluation (CPU BASELINE ONLY; see
    orc_bpr_hogwild_epoch).  U/I/bias updated in place.  Returns (t_update, t_eval, loss)."""
    for a in (U, I, bias):
        assert a.dtype == np.float64 and a.flags.c_contiguous
    pu = np.ascontiguousarray(pos_user, np.int64)
    pi = np.ascontiguousarray(pos_item, np.int64)
    ev = np.ascontiguousarray(eval_set, np.int64)
    out = np.zeros(3, np.float64)
    rc = lib().orc_bpr_hogwild_epoch(_p(U, c_f64p), _p(I, c_f64p), _p(bias, c_f64p), U.shape[1],
                                     _p(pu, c_i64p), _p(pi, c_i64p), len(pu), U.shape[0],
                                     int(nitems), int(num_neg), int(nthreads), int(seed),
                                     lr, bias_lambda, user_lambda, item_lambda, int(use_biases),
                                     _p(ev, c_i64p), len(ev), _p(out[0:], c_f64p),
                                     _p(out[1:], c_f64p), _p(out[2:], c_f64p))
    if rc:
        raise RuntimeError("gradients too big")
    return float(out[0]), float(out[1]), float(out[2])


def bpr_sets(users, items, values, test=None, eval_num_neg=3, eval_seed=42):
    """BPREngine::init/initTest bookkeeping (BPREngine.cpp:63-131): (uids, iids, evalSet,
    testEvalSet) with triplets as int64 (n, 3) arrays."""
    u = np.ascontiguousarray(users, np.int64)
    i = np.ascontiguousarray(items, np.int64)
    v = np.ascontiguousarray(values, np.float64)
    if test is None:
        test = (np.zeros(0, np.int64), np.zeros(0, np.int64), np.zeros(0))
    tu = np.ascontiguousarray(test[0], np.int64)
    ti = np.ascontiguousarray(test[1], np.int64)
    tv = np.ascontiguousarray(test[2], np.float64)
    n, tn = len(u), len(tu)
    nu, ni, ne, nt = (ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64())
    uids = np.zeros(max(n, 1), np.int64)
    iids = np.zeros(max(n, 1), np.int64)
    ev = np.zeros((max(n * eval_num_neg, 1), 3), np.int64)
    tev = np.zeros((max(tn * eval_num_neg, 1), 3), np.int64)
    rc = lib().orc_bpr_sets(_p(u, c_i64p), _p(i, c_i64p), _p(v, c_f64p), n, _p(tu, c_i64p),
                            _p(ti, c_i64p), _p(tv, c_f64p), tn, eval_num_neg, eval_seed,
                            ctypes.byref(nu), ctypes.byref(ni), _p(uids, c_i64p),
                            _p(iids, c_i64p), _p(ev, c_i64p), ctypes.byref(ne),
                            _p(tev, c_i64p), ctypes.byref(nt))
    if rc:
        raise ValueError("a user has every item as a positive")
    return uids[:nu.value], iids[:ni.value], ev[:ne.value], tev[:nt.value]


# ---- test-set evaluation (numpy restatement; test infrastructure) ---------------------------
def test_scores(U, I, users, bias=None):
    """Engine::computeTestScores (Engine.cpp:73-96): score = bias_i (or 0), then += u_f·q_f in
    factor order.  numpy's elementwise multiply and add round each step like the reference's
    double loop (no fused multiply-add), so the scores are the reference's bit for bit."""
    U = np.asarray(U, np.float64)
    I = np.asarray(I, np.float64)
    out = np.empty((len(users), I.shape[0]))
    for t, u in enumerate(users):
        s = np.zeros(I.shape[0]) if bias is None else np.array(bias, np.float64)
        for f in range(I.shape[1]):
            s = s + U[u, f] * I[:, f]
        out[t] = s
    return out


def _sorted_pairs(labels, scores):
    # (score, label > 0) pairs sorted descending as std::greater<pair<Double, bool>>
    pos = np.asarray(labels) > 0.0
    order = np.lexsort((pos, np.asarray(scores)))[::-1]
    return pos[order]


def metric_mse(labels, scores):
    """MeanSquaredError::compute, Metrics.cpp:59-69 (sequential sum: cumsum)."""
    d = np.asarray(labels, np.float64) - np.asarray(scores, np.float64)
    assert len(d) > 0
    return np.cumsum(d * d)[-1] / len(d)


def metric_auc(labels, scores):
    """AUC::compute, Metrics.cpp:71-106: each negative adds tp/pos/neg in sorted order."""
    p = _sorted_pairs(labels, scores)
    pos = int(p.sum())
    neg = len(p) - pos
    if pos == 0 or neg == 0:
        return 1.0
    tp = np.cumsum(p)
    terms = tp[~p].astype(np.float64) / pos / neg
    return float(np.cumsum(terms)[-1]) if len(terms) else 0.0


def metric_precision(labels, scores, k):
    """Precision::compute, Metrics.cpp:108-122 (positives among the k best pairs)."""
    assert len(labels) >= k
    return float(_sorted_pairs(labels, scores)[:k].sum()) / k


def metric_recall(labels, scores, k):
    """Recall::compute, Metrics.cpp:124-145."""
    assert len(labels) >= k
    p = _sorted_pairs(labels, scores)
    assert p.sum() > 0
    return float(p[:k].sum()) / int(p.sum())


def metric_ap(labels, scores):
    """AveragePrecision::compute, Metrics.cpp:147-163."""
    p = _sorted_pairs(labels, scores)
    tot = int(p.sum())
    assert tot > 0
    r = np.nonzero(p)[0]
    terms = np.arange(1, tot + 1, dtype=np.float64) / (r + 1)
    return float(np.cumsum(terms)[-1]) / tot


def rank_stats(labels, scores):
    """What qmfx_eval_ranks returns for one user, by brute force: Σ score², and per positive
    (label > 0, item order) its score and the count of items scored strictly higher."""
    labels = np.asarray(labels)
    scores = np.asarray(scores)
    pi = np.nonzero(labels > 0)[0]
    above = np.array([np.count_nonzero(scores > scores[i]) for i in pi], np.int64)
    return float(np.sum(scores * scores)), scores[pi], above
