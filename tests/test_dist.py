"""Multi-GPU decomposition, rehearsed on CPU with torch.distributed gloo (world_size 2, 3, 4
and 8, uniform and power-law data — the latter with empty pieces and ranks): each rank solves its nnz-balanced contiguous row range (qmfx_partition_rows, the
product's partitioner), split into the product's solve pieces (qmfx_dist_plan, the same
code qmfx_wals_half runs), solved piece by piece (the oracle stands in for the device
solve), each piece broadcast by its owner and the loss all-reduced — the exchange
qmfx_wals_half does with RCCL (grouped ncclBroadcast per piece and rank + ncclAllReduce,
DESIGN.md §6).  The assembled
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


def _data(kind="uniform"):
    if kind == "uniform":
        u, i, v = synth(1500, 400, 20000, seed=21)
    else:
        # power-law rows: a few users and items hold most signals, so nnz-balanced ranges are
        # ragged and, at 8 ranks × 8 pieces, some pieces and whole ranks are empty
        rng = np.random.default_rng(22)
        n = 20000
        u = np.minimum((rng.pareto(0.7, n) * 3).astype(np.int64), 1499)
        i = np.minimum((rng.pareto(0.7, n) * 2).astype(np.int64), 399)
        key = np.unique(u * 400 + i)
        u, i = key // 400, key % 400
        v = rng.integers(1, 6, len(u)).astype(np.float64)
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


P = 8  # solve pieces per rank (qmfx_wals_half's default with several ranks, QMFX_PIECES)


def _worker(rank, world, port, result_q, kind="uniform"):
    """One rank of qmfx_wals_half's multi-GPU schedule: for each piece j, solve this rank's
    rows of piece j, then every rank r broadcasts its piece-j rows (skipped when empty) —
    the grouped ncclBroadcast loop, here over gloo; then the loss all-reduce."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        u, i, v, uids, iids, ucsr, icsr, init = _data(kind)
        nu, ni = len(uids), len(iids)
        out = {}
        fixed = init
        for side, csr, n, n_other in ((0, ucsr, nu, ni), (1, icsr, ni, nu)):
            plan = qmf_amd.dist_plan(csr[0], world, P)
            replica = np.full((n, K), np.nan)  # every row must be written by the exchange
            sends = np.zeros(n, np.int64)
            loss = 0.0
            for j in range(P):
                b, e = int(plan[rank, j]), int(plan[rank, j + 1])
                if e > b:
                    local, l = _solve_range(side, csr, n_other, fixed, b, e)
                    replica[b:e] = local
                    loss += l
                for r in range(world):
                    rb, re = int(plan[r, j]), int(plan[r, j + 1])
                    if re <= rb:
                        continue
                    t = torch.from_numpy(np.ascontiguousarray(replica[rb:re]))
                    dist.broadcast(t, src=r)
                    replica[rb:re] = t.numpy()
                    sends[rb:re] += 1
            t = torch.tensor([loss], dtype=torch.float64)
            dist.all_reduce(t)
            b, e = qmf_amd.partition_rows(csr[0], world, rank)
            empty = sum(int(plan[rank, j + 1] == plan[rank, j]) for j in range(P))
            out[side] = (replica, float(t[0]) / (nu * ni), int(csr[0][e] - csr[0][b]), sends,
                         empty)
            fixed = replica
        result_q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_plan_covers_rows_once_in_owner_order():
    """qmfx_dist_plan: per rank, P contiguous pieces inside the rank's partition_rows range;
    over all ranks every row exactly once, ascending; empty ranks/pieces allowed."""
    for rp in (np.array([0, 5, 5, 9, 30, 31]), np.array([0, 1000]), np.array([0, 0, 0, 0]),
               np.concatenate([[0], np.cumsum(np.random.default_rng(1).integers(0, 50, 997))])):
        for world in (1, 2, 3, 8):
            plan = qmf_amd.dist_plan(rp, world, P)
            n = len(rp) - 1
            assert plan[0, 0] == 0 and plan[-1, -1] == n
            flat = plan[:, :].ravel()
            assert np.all(np.diff(flat) >= 0)  # ascending: pieces and ranks in row order
            for r in range(world):
                assert tuple(qmf_amd.partition_rows(rp, world, r)) == (plan[r, 0], plan[r, -1])
                if r + 1 < world:
                    assert plan[r, -1] == plan[r + 1, 0]


@pytest.mark.parametrize("world,kind", [(2, "uniform"), (3, "uniform"), (4, "uniform"),
                                        (8, "uniform"), (4, "skewed"), (8, "skewed")])
def test_sharded_half_epochs_equal_single_process(world, kind):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, kind)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    u, i, v, uids, iids, ucsr, icsr, init = _data(kind)
    o = po.OracleWALS(u, i, v, K, LAM, ALPHA)
    o.set_factors(1, init)
    ref = {}
    for side in (0, 1):
        ref[side] = (o.iterate(side), o.factors(side))
    for r in range(world):
        for side in (0, 1):
            full, loss, _, sends, _ = res[r][side]
            # every row arrived exactly once per half (from its owner's broadcast) ...
            assert np.all(sends == 1), (r, side)
            # ... and every rank holds the same complete factor matrix as 1 process
            assert np.array_equal(full, ref[side][1]), (r, side)
            assert abs(loss - ref[side][0]) <= 1e-12 * abs(ref[side][0])
    if kind == "uniform":
        # the shards are nnz-balanced
        for side in (0, 1):
            loads = [res[r][side][2] for r in range(world)]
            assert max(loads) - min(loads) <= 0.05 * sum(loads)
    else:
        # the skewed data really exercises empty pieces (and the exchange skips them)
        assert sum(res[r][side][4] for r in range(world) for side in (0, 1)) > 0
