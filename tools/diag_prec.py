"""fp32 parity diagnostic (GPU): per-half and multi-epoch factor errors of the fp32 device
path against the oracle at the reference's lambda=0.05, alpha=40, by row route."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import pyoracle as po  # noqa: E402
import qmf_amd  # noqa: E402
from helpers import csr_from_triples, load_ml100k, rel_err, synth  # noqa: E402

LAM, ALPHA = 0.05, 40.0
NT = 16


def pair(u, i, v, k, prec, init):
    o = po.OracleWALS(u, i, v, k, LAM, ALPHA)
    uids, iids, (urp, ucol, uval), (irp, icol, ival) = csr_from_triples(u, i, v)
    c = qmf_amd.Context(k, prec)
    c.set_shape(len(uids), len(iids))
    c.upload_csr(0, urp, ucol, uval)
    c.upload_csr(1, irp, icol, ival)
    o.set_factors(1, init)
    c.set_factors(1, init)
    return o, c


def lockstep(name, u, i, v, k, halves=4, prec=32):
    rng = np.random.default_rng(1)
    init = rng.uniform(-0.01, 0.01, (len(np.unique(i)), k))
    o, c = pair(u, i, v, k, prec, init)
    out = []
    for h in range(halves):
        side = h % 2
        t0 = time.time()
        lo = o.iterate(side, NT)
        ld = c.wals_half(side, ALPHA, LAM) / (o.nusers * o.nitems)
        e = rel_err(c.factors(side), o.factors(side))
        out.append("h%d side%d err %.2e loss %.2e (%.1fs)" % (h, side, e, abs(ld - lo) / abs(lo), time.time() - t0))
        c.set_factors(side, o.factors(side))
    print(name, "|", "; ".join(out), flush=True)


def independent(name, u, i, v, k, init, epochs, prec=32):
    o, c = pair(u, i, v, k, prec, init)
    out = []
    for ep in range(epochs):
        o.iterate(0, NT)
        c.wals_half(0, ALPHA, LAM)
        o.iterate(1, NT)
        c.wals_half(1, ALPHA, LAM)
        out.append("%.1e/%.1e" % (rel_err(c.factors(0), o.factors(0)), rel_err(c.factors(1), o.factors(1))))
    print(name, "| U/I per epoch:", " ".join(out), flush=True)


def main():
    d = load_ml100k()
    k = 30
    init = d["init"][: 1682 * k].reshape(1682, k)
    for nw in ("0", "1"):
        os.environ["QMFX_NO_WHITEN"] = nw
        independent("ml100k k30 nowhiten=%s" % nw, d["users"], d["items"], d["values"], k, init, 10)
        lockstep("ml100k k30 lockstep nowhiten=%s" % nw, d["users"], d["items"], d["values"], k)
    u, i, v = synth(20000, 2000, 1_000_000, seed=1)
    for k in (64, 128, 256):
        for nw in ("0", "1"):
            os.environ["QMFX_NO_WHITEN"] = nw
            lockstep("c2shape k%d nowhiten=%s" % (k, nw), u, i, v, k)
    os.environ["QMFX_NO_WHITEN"] = "0"
    u, i, v = synth(12000, 60, 30000, seed=96)
    lockstep("degenerate 12000x60 k96", u, i, v, 96, halves=2)


if __name__ == "__main__":
    main()
