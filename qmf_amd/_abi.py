"""ctypes bindings for libqmfx.so (include/qmfx.h)."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("QMFX_LIB") or os.path.join(_HERE, "_build", "libqmfx.so")

c_i64 = ctypes.c_int64
c_u64 = ctypes.c_uint64
c_int = ctypes.c_int
c_dbl = ctypes.c_double
vp = ctypes.c_void_p
P_i64 = ctypes.POINTER(c_i64)
P_i32 = ctypes.POINTER(ctypes.c_int32)
P_f64 = ctypes.POINTER(c_dbl)
P_f32 = ctypes.POINTER(ctypes.c_float)
P_u8 = ctypes.POINTER(ctypes.c_uint8)
P_int = ctypes.POINTER(c_int)

# name -> argtypes (all return int status unless listed in _RESTYPE)
SIGNATURES = {
    "qmfx_last_error": [],
    "qmfx_version": [],
    "qmfx_device_count": [P_int],
    "qmfx_create": [ctypes.POINTER(vp), c_int, c_int, c_int],
    "qmfx_destroy": [vp],
    "qmfx_sync": [vp],
    "qmfx_set_shape": [vp, c_i64, c_i64],
    "qmfx_get_shape": [vp, P_i64, P_i64, P_i64],
    "qmfx_upload_csr": [vp, c_int, P_i64, P_i32, P_f64, c_i64],
    "qmfx_gen_synthetic": [vp, c_i64, c_i64, c_i64, c_u64, P_i64],
    "qmfx_gen_synthetic_zipf": [vp, c_i64, c_i64, c_i64, c_u64, c_dbl, P_i64],
    "qmfx_download_csr": [vp, c_int, P_i64, P_i32, P_f64],
    "qmfx_group_signals": [vp, vp, c_i64, P_i64, P_i64],
    "qmfx_get_ids": [vp, c_int, P_i64],
    "qmfx_import_signals": [vp, vp],
    "qmfx_set_factors": [vp, c_int, P_f64],
    "qmfx_get_factors": [vp, c_int, P_f64],
    "qmfx_fill_uniform": [vp, c_int, c_dbl, c_u64],
    "qmfx_wals_half": [vp, c_int, c_dbl, c_dbl, P_f64],
    "qmfx_wals_failed_rows": [vp, P_i64, c_i64, P_i64],
    "qmfx_wals_row_losses": [vp, P_f64],
    "qmfx_row_classes": [vp, c_int, P_i64],
    "qmfx_wals_row_system": [vp, c_int, c_i64, c_dbl, c_dbl, P_f64, P_f64, P_f64],
    "qmfx_wals_set_row": [vp, c_int, c_i64, P_f64],
    "qmfx_bpr_set_positives": [vp, P_i64, P_i64, c_i64],
    "qmfx_bpr_set_biases": [vp, P_f64],
    "qmfx_bpr_get_biases": [vp, P_f64],
    "qmfx_bpr_epoch": [vp, c_u64, c_int, c_dbl, c_dbl, c_dbl, c_dbl, c_int, c_int],
    "qmfx_bpr_apply": [vp, P_i64, c_i64, c_dbl, c_dbl, c_dbl, c_dbl, c_int],
    "qmfx_bpr_eval": [vp, c_int, P_i64, c_i64, c_int, P_f64],
    "qmfx_eval_set_labels": [vp, c_i64, P_i64, P_i64, P_i64, P_f64],
    "qmfx_eval_ranks": [vp, c_int, P_f64, P_i64, P_f64],
    "qmfx_rccl_unique_id": [P_u8],
    "qmfx_dist_init": [vp, c_int, c_int, P_u8],
    "qmfx_partition_rows": [P_i64, c_i64, c_int, c_int, P_i64, P_i64],
    "qmfx_dist_plan": [P_i64, c_i64, c_int, c_int, P_i64],
    "qmfx_dist_init_all": [ctypes.POINTER(vp), c_int],
    "qmfx_wals_half_multi": [ctypes.POINTER(vp), c_int, c_int, c_dbl, c_dbl, P_f64],
    "qmfx_solve_kernel_stats": [vp, P_f64, P_i64, P_f64, P_f64],
    "qmfx_kernel_stats": [vp, c_int, P_f64, P_i64, P_f64, P_f64],
    "qmfx_kernel_stats_side": [vp, c_int, c_int, P_f64, P_i64, P_f64, P_f64],
    "qmfx_reset_stats": [vp],
    "qmfx_exchange_stats": [vp, c_int, P_f64, P_f64, P_f64, P_i64],
    "qmfx_bpr_plan": [vp, P_int, P_int],
    "qmfx_build_variant": [],
    "qmfx_selftest_mfma": [c_int, c_int, P_f64, P_f64, P_f64],
}
_RESTYPE = {"qmfx_last_error": ctypes.c_char_p, "qmfx_build_variant": ctypes.c_char_p}

_lib = None


class QmfxError(RuntimeError):
    pass


def build():
    subprocess.run(["make", "-s", "-C", _HERE, "-j8"], check=True)


def lib():
    """Loads libqmfx.so.  Raises if it has not been built (no silent fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise QmfxError("libqmfx.so not built (%s): run `make -C qmf_amd` or "
                            "__graft_entry__.build()" % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        for name, argt in SIGNATURES.items():
            fn = getattr(L, name)
            fn.argtypes = argt
            fn.restype = _RESTYPE.get(name, c_int)
        _lib = L
    return _lib


def _check(rc):
    if rc != 0:
        raise QmfxError("qmfx error %d: %s" % (rc, lib().qmfx_last_error().decode()))


def _p(a, t):
    return a.ctypes.data_as(t)


def version():
    return lib().qmfx_version()


def build_variant():
    """'' for the product library; the compile flags of a timing-variant build."""
    return lib().qmfx_build_variant().decode()


def selftest_mfma(precision, A, B, device=0):
    A = np.ascontiguousarray(A, np.float64)
    B = np.ascontiguousarray(B, np.float64)
    C = np.zeros((16, 16), np.float64)
    _check(lib().qmfx_selftest_mfma(device, precision, _p(A, P_f64), _p(B, P_f64), _p(C, P_f64)))
    return C


def device_count():
    """Visible HIP devices (initialises the HIP runtime in this process)."""
    n = c_int(0)
    _check(lib().qmfx_device_count(ctypes.byref(n)))
    return n.value


def rccl_unique_id():
    buf = (ctypes.c_uint8 * 128)()
    _check(lib().qmfx_rccl_unique_id(buf))
    return bytes(buf)


def partition_rows(rowptr, world, rank):
    rp = np.ascontiguousarray(rowptr, np.int64)
    b = c_i64(0)
    e = c_i64(0)
    _check(lib().qmfx_partition_rows(_p(rp, P_i64), len(rp) - 1, world, rank, ctypes.byref(b),
                                     ctypes.byref(e)))
    return b.value, e.value


def dist_plan(rowptr, world, npieces):
    """[world][npieces + 1] piece boundaries of the half-epoch all-gather schedule."""
    rp = np.ascontiguousarray(rowptr, np.int64)
    out = np.zeros((world, npieces + 1), np.int64)
    _check(lib().qmfx_dist_plan(_p(rp, P_i64), len(rp) - 1, world, npieces, _p(out, P_i64)))
    return out


def dist_init_all(ctxs):
    """One process, several GPUs: the contexts (one per device, rank order) become one RCCL
    clique (qmfx_dist_init_all)."""
    arr = (vp * len(ctxs))(*[c.h for c in ctxs])
    _check(lib().qmfx_dist_init_all(arr, len(ctxs)))


def wals_half_multi(ctxs, side, alpha, lam):
    """qmfx_wals_half over every context of one dist_init_all; returns the global loss sum."""
    arr = (vp * len(ctxs))(*[c.h for c in ctxs])
    out = c_dbl(0)
    _check(lib().qmfx_wals_half_multi(arr, len(ctxs), side, alpha, lam, ctypes.byref(out)))
    return out.value


class Context:
    """One device context (one GPU).  Mirrors the device state of a WALSEngine/BPREngine."""

    def __init__(self, nfactors, precision=64, device=0):
        L = lib()
        h = vp()
        _check(L.qmfx_create(ctypes.byref(h), device, precision, nfactors))
        self.h = h
        self.k = nfactors
        self.precision = precision
        self.nusers = 0
        self.nitems = 0

    def close(self):
        if getattr(self, "h", None):
            lib().qmfx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ---- data
    def set_shape(self, nusers, nitems):
        _check(lib().qmfx_set_shape(self.h, nusers, nitems))
        self.nusers, self.nitems = nusers, nitems

    def upload_csr(self, side, rowptr, colidx, values):
        rp = np.ascontiguousarray(rowptr, np.int64)
        col = np.ascontiguousarray(colidx, np.int32)
        val = np.ascontiguousarray(values, np.float64)
        _check(lib().qmfx_upload_csr(self.h, side, _p(rp, P_i64), _p(col, P_i32), _p(val, P_f64),
                                     len(col)))

    def gen_synthetic(self, nusers, nitems, nnz, seed):
        out = c_i64(0)
        _check(lib().qmfx_gen_synthetic(self.h, nusers, nitems, nnz, seed, ctypes.byref(out)))
        self.nusers, self.nitems = nusers, nitems
        return out.value

    def gen_synthetic_zipf(self, nusers, nitems, ndraws, seed, zipf_s):
        """Power-law item popularity (qmfx_gen_synthetic_zipf); returns the unique nnz."""
        out = c_i64(0)
        _check(lib().qmfx_gen_synthetic_zipf(self.h, nusers, nitems, ndraws, seed, float(zipf_s),
                                             ctypes.byref(out)))
        self.nusers, self.nitems = nusers, nitems
        return out.value

    def group_signals(self, users, items, values):
        """Device ingest (qmfx_group_signals) of raw (user id, item id, value) triples in
        file order; returns (user ids, item ids), ascending."""
        rec = np.empty(len(users), dtype=np.dtype([("u", "<i8"), ("i", "<i8"), ("v", "<f8")]))
        rec["u"], rec["i"], rec["v"] = users, items, values
        nu, ni = c_i64(0), c_i64(0)
        _check(lib().qmfx_group_signals(self.h, rec.ctypes.data_as(vp), len(rec),
                                        ctypes.byref(nu), ctypes.byref(ni)))
        self.nusers, self.nitems = nu.value, ni.value
        return self.ids(0), self.ids(1)

    def import_signals(self, src):
        """Take src's shape, ids and both CSRs device to device (qmfx_import_signals)."""
        _check(lib().qmfx_import_signals(self.h, src.h))
        self.nusers, self.nitems, _ = self.shape()

    def ids(self, side):
        out = np.empty(self.nusers if side == 0 else self.nitems, np.int64)
        _check(lib().qmfx_get_ids(self.h, side, _p(out, P_i64)))
        return out

    def shape(self):
        a, b, c = c_i64(), c_i64(), c_i64()
        _check(lib().qmfx_get_shape(self.h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
        return a.value, b.value, c.value

    def download_csr(self, side):
        nu, ni, nnz = self.shape()
        n = nu if side == 0 else ni
        rp = np.empty(n + 1, np.int64)
        col = np.empty(max(nnz, 1), np.int32)
        val = np.empty(max(nnz, 1), np.float64)  # exactly the device's values (fp32 widened)
        _check(lib().qmfx_download_csr(self.h, side, _p(rp, P_i64), _p(col, P_i32), _p(val, P_f64)))
        return rp, col[:nnz], val[:nnz]

    # ---- factors
    def _n(self, side):
        return self.nusers if side == 0 else self.nitems

    def set_factors(self, side, F):
        F = np.ascontiguousarray(F, np.float64)
        assert F.shape == (self._n(side), self.k), F.shape
        _check(lib().qmfx_set_factors(self.h, side, _p(F, P_f64)))

    def factors(self, side):
        out = np.empty((self._n(side), self.k), np.float64)
        _check(lib().qmfx_get_factors(self.h, side, _p(out, P_f64)))
        return out

    def fill_uniform(self, side, bound, seed):
        _check(lib().qmfx_fill_uniform(self.h, side, bound, seed))

    # ---- WALS
    def wals_half(self, side, alpha, lam):
        out = c_dbl(0)
        _check(lib().qmfx_wals_half(self.h, side, alpha, lam, ctypes.byref(out)))
        return out.value

    def row_classes(self, side):
        """Row plan of a side: {'whitened': [8 bucket counts], 'direct', 'heavy', 'segments'}."""
        out = np.zeros(11, np.int64)
        _check(lib().qmfx_row_classes(self.h, side, _p(out, P_i64)))
        return {"whitened": out[:8].tolist(), "direct": int(out[8]), "heavy": int(out[9]),
                "segments": int(out[10])}

    def row_losses(self, side):
        out = np.empty(self._n(side), np.float64)
        _check(lib().qmfx_wals_row_losses(self.h, _p(out, P_f64)))
        return out

    def failed_rows(self):
        cnt = c_i64(0)
        _check(lib().qmfx_wals_failed_rows(self.h, None, 0, ctypes.byref(cnt)))
        rows = np.empty(max(cnt.value, 1), np.int64)
        _check(lib().qmfx_wals_failed_rows(self.h, _p(rows, P_i64), cnt.value, ctypes.byref(cnt)))
        return rows[: cnt.value]

    def row_system(self, side, row, alpha, lam):
        """(A, b, Σc) of one row's k×k system, built on the device."""
        k = self.k
        A = np.empty((k, k), np.float64)
        b = np.empty(k, np.float64)
        cs = np.zeros(1, np.float64)
        _check(lib().qmfx_wals_row_system(self.h, side, int(row), float(alpha), float(lam),
                                          _p(A, P_f64), _p(b, P_f64), _p(cs, P_f64)))
        return A, b, float(cs[0])

    def sync(self):
        _check(lib().qmfx_sync(self.h))

    # ---- BPR
    def bpr_set_positives(self, users, items):
        u = np.ascontiguousarray(users, np.int64)
        i = np.ascontiguousarray(items, np.int64)
        _check(lib().qmfx_bpr_set_positives(self.h, _p(u, P_i64), _p(i, P_i64), len(u)))

    def bpr_set_biases(self, b):
        b = np.ascontiguousarray(b, np.float64)
        _check(lib().qmfx_bpr_set_biases(self.h, _p(b, P_f64)))

    def bpr_biases(self):
        out = np.empty(self.nitems, np.float64)
        _check(lib().qmfx_bpr_get_biases(self.h, _p(out, P_f64)))
        return out

    def bpr_epoch(self, seed, num_neg, lr, bias_lambda, user_lambda, item_lambda, use_biases,
                  shuffle=True):
        _check(lib().qmfx_bpr_epoch(self.h, seed, num_neg, lr, bias_lambda, user_lambda,
                                    item_lambda, int(use_biases), int(shuffle)))

    def bpr_apply(self, triplets, lr, bias_lambda, user_lambda, item_lambda, use_biases):
        t = np.ascontiguousarray(triplets, np.int64).reshape(-1, 3)
        _check(lib().qmfx_bpr_apply(self.h, _p(t, P_i64), len(t), lr, bias_lambda, user_lambda,
                                    item_lambda, int(use_biases)))

    def bpr_eval(self, slot, triplets, use_biases):
        t = np.ascontiguousarray(triplets, np.int64).reshape(-1, 3)
        self._keep_trip = getattr(self, "_keep_trip", {})
        self._keep_trip[slot] = t
        out = c_dbl(0)
        _check(lib().qmfx_bpr_eval(self.h, slot, _p(t, P_i64), len(t), int(use_biases),
                                   ctypes.byref(out)))
        return out.value

    # ---- test-set evaluation (Engine.cpp:73-96, Metrics.cpp:27-164)
    def eval_set_labels(self, users, rowptr, items, values):
        """Test users (user idx) and their labelled items as a CSR over the test slots."""
        users = np.ascontiguousarray(users, np.int64)
        rowptr = np.ascontiguousarray(rowptr, np.int64)
        items = np.ascontiguousarray(items, np.int64)
        values = np.ascontiguousarray(values, np.float64)
        if len(rowptr) != len(users) + 1 or len(items) != rowptr[-1] or len(values) != len(items):
            raise QmfxError("label CSR shape mismatch")
        _check(lib().qmfx_eval_set_labels(self.h, len(users), _p(users, P_i64), _p(rowptr, P_i64),
                                          _p(items, P_i64), _p(values, P_f64)))
        self._ev = (len(users), int(rowptr[-1]), int(np.count_nonzero(values > 0)))

    def eval_ranks(self, use_biases=False):
        """(label_scores, above, sq_sum): see include/qmfx.h qmfx_eval_ranks."""
        nt, nl, npos = self._ev
        ls, ab, sq = np.empty(nl), np.empty(npos, np.int64), np.empty(nt)
        _check(lib().qmfx_eval_ranks(self.h, int(use_biases), _p(ls, P_f64), _p(ab, P_i64),
                                     _p(sq, P_f64)))
        return ls, ab, sq

    # ---- dist / stats
    def dist_init(self, rank, world, uid):
        """uid = rank 0's rccl_unique_id(), or None: partition and shard without a
        communicator (each half solves only this rank's rows)."""
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(uid) if uid is not None else None
        _check(lib().qmfx_dist_init(self.h, rank, world, buf))

    def solve_stats(self):
        ms, n, fl, by = c_dbl(), c_i64(), c_dbl(), c_dbl()
        _check(lib().qmfx_solve_kernel_stats(self.h, ctypes.byref(ms), ctypes.byref(n),
                                             ctypes.byref(fl), ctypes.byref(by)))
        return dict(ms=ms.value, launches=n.value, flops=fl.value, bytes=by.value)

    def kernel_stats(self, cls):
        ms, n, fl, by = c_dbl(), c_i64(), c_dbl(), c_dbl()
        _check(lib().qmfx_kernel_stats(self.h, cls, ctypes.byref(ms), ctypes.byref(n),
                                       ctypes.byref(fl), ctypes.byref(by)))
        return dict(ms=ms.value, launches=n.value, flops=fl.value, bytes=by.value)

    def kernel_stats_side(self, cls, side):
        """kernel_stats(cls) over the halves that solved `side` only."""
        ms, n, fl, by = c_dbl(), c_i64(), c_dbl(), c_dbl()
        _check(lib().qmfx_kernel_stats_side(self.h, cls, side, ctypes.byref(ms), ctypes.byref(n),
                                            ctypes.byref(fl), ctypes.byref(by)))
        return dict(ms=ms.value, launches=n.value, flops=fl.value, bytes=by.value)

    def reset_stats(self):
        _check(lib().qmfx_reset_stats(self.h))

    def exchange_stats(self, side):
        """Multi-rank halves that solved `side` since reset (include/qmfx.h
        qmfx_exchange_stats): exchange_ms, exposed_ms, solve_ms (sums) and halves."""
        x, t, sv, n = c_dbl(), c_dbl(), c_dbl(), c_i64()
        _check(lib().qmfx_exchange_stats(self.h, side, ctypes.byref(x), ctypes.byref(t),
                                         ctypes.byref(sv), ctypes.byref(n)))
        return dict(exchange_ms=x.value, exposed_ms=t.value, solve_ms=sv.value, halves=n.value)

    def bpr_plan(self):
        """(waves, atomic_user) of the last bpr_epoch."""
        w, a = c_int(), c_int()
        _check(lib().qmfx_bpr_plan(self.h, ctypes.byref(w), ctypes.byref(a)))
        return w.value, a.value
