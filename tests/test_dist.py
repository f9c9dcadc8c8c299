"""Multi-GPU decomposition, rehearsed on CPU with torch.distributed gloo (world_size 2 and
3): each rank solves its nnz-balanced contiguous row range (qmfx_partition_rows, the
product's partitioner; the oracle stands in for the device solve), the solved ranges are
all-gathered and the loss all-reduced — the exchange qmfx_wals_half does with RCCL
(grouped ncclBroadcast per rank range + ncclAllReduce).  The assembled
factors must equal the single-process solve bit for bit (rows are independent given the
fixed side), and the loss to rounding."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import pyoracle as po
import qmf_amd
from helpers import csr_from_triples, synth

K, LAM, ALPHA = 16, 0.05, 40.0


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _data():
    u, i, v = synth(1500, 400, 20000, seed=21)
    uids, iids, ucsr, icsr = csr_from_triples(u, i, v)
    init = np.random.default_rng(3).uniform(-0.01, 0.01, (len(iids), K))
    return u, i, v, uids, iids, ucsr, icsr, init


def _solve_range(side, csr, n_other, fixed, b, e):
    """Rows [b, e) of `side` with the other side fixed (oracle sub-problem); returns the
    solved rows and their loss SUM."""
    rp, col, val = csr
    srp = (rp[b:e + 1] - rp[b]).astype(np.int64)
    scol = col[rp[b]:rp[e]]
    sval = val[rp[b]:rp[e]]
    empty = (np.zeros(n_other + 1, np.int64), np.zeros(1, np.int32), np.zeros(1, np.float32))
    empty_rows = (np.zeros(e - b + 1, np.int64), np.zeros(1, np.int32), np.zeros(1, np.float32))
    if side == 0:
        o = po.OracleWALS.from_csr(e - b, n_other, srp, scol, sval, *empty, K, LAM, ALPHA)
    else:
        o = po.OracleWALS.from_csr(n_other, e - b, *empty, srp, scol, sval, K, LAM, ALPHA)
    o.set_factors(1 - side, fixed)
    loss = o.iterate(side) * (e - b) * n_other
    return o.factors(side), loss


def _allgather_rows(local, b, e, n, world):
    """All-gather-v of contiguous row ranges (what the grouped broadcasts do)."""
    counts = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(counts, torch.tensor([b, e], dtype=torch.int64))
    mx = max(int(c[1] - c[0]) for c in counts)
    buf = torch.zeros((mx, local.shape[1]), dtype=torch.float64)
    buf[: e - b] = torch.from_numpy(local)
    bufs = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(bufs, buf)
    out = np.zeros((n, local.shape[1]))
    for c, t in zip(counts, bufs):
        cb, ce = int(c[0]), int(c[1])
        out[cb:ce] = t[: ce - cb].numpy()
    return out


def _worker(rank, world, port, result_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        u, i, v, uids, iids, ucsr, icsr, init = _data()
        nu, ni = len(uids), len(iids)
        out = {}
        fixed = init
        for side, csr, n, n_other in ((0, ucsr, nu, ni), (1, icsr, ni, nu)):
            b, e = qmf_amd.partition_rows(csr[0], world, rank)
            local, loss = _solve_range(side, csr, n_other, fixed, b, e)
            full = _allgather_rows(local, b, e, n, world)
            t = torch.tensor([loss], dtype=torch.float64)
            dist.all_reduce(t)
            out[side] = (full, float(t[0]) / (nu * ni), int(csr[0][e] - csr[0][b]))
            fixed = full
        result_q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_half_epochs_equal_single_process(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    u, i, v, uids, iids, ucsr, icsr, init = _data()
    o = po.OracleWALS(u, i, v, K, LAM, ALPHA)
    o.set_factors(1, init)
    ref = {}
    for side in (0, 1):
        ref[side] = (o.iterate(side), o.factors(side))
    for r in range(world):
        for side in (0, 1):
            full, loss, _ = res[r][side]
            # every rank holds the same, complete factor matrix, equal to the 1-process one
            assert np.array_equal(full, ref[side][1]), (r, side)
            assert abs(loss - ref[side][0]) <= 1e-12 * abs(ref[side][0])
    # the shards are nnz-balanced
    for side in (0, 1):
        loads = [res[r][side][2] for r in range(world)]
        assert max(loads) - min(loads) <= 0.05 * sum(loads)
