"""WALS throughput benchmark on MI355X (BASELINE.json metric: solves/s and ms/epoch at
k=128, with the achieved roofline fraction of the dominant kernel).

A "step" is one WALS epoch (user half + item half, WALSEngine::optimize's loop body,
WALSEngine.cpp:82-96) over a synthetic interaction matrix resident in HBM.  Default
workload: BASELINE configs[2] (10M users × 1M items, 500M nnz, k=128) at the reference's
precision, fp64 (qmf/Types.h:24; the drop-in CLIs default to it too) — the largest k=128
configuration, which fits one GPU.  `--config c3z` is the same shape with Zipf(1.0) item
popularity (SURVEY.md §8(d) skew variant: power-law rows of up to ~10M signals).

`--gpus N` runs N ranks: without a torch.distributed launcher in the environment it
re-launches itself under `torch.distributed.run` as a child process (before anything touches
the GPU); each rank then takes one GPU, the matrix is split over the ranks by nnz-balanced
row ranges and each half ends with an RCCL all-gather of the solved factors (strong
scaling: total work fixed).  A rank count that does not match --gpus, or more ranks than
visible GPUs, fails with a non-zero exit.

The CPU baseline (rank 0, N=1) is one full epoch of the reference-structure port on the box's
CPU share (BASELINE.md CPU-baseline plan: "C3 and C5: time >= 1 full epoch"); when the time
guard predicts that the epoch would not finish inside the run's time limit it falls back to
the sampled estimate and says so.

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (nusers, nitems, nnz, k, seed)
    "c3": (10_000_000, 1_000_000, 500_000_000, 128, 3),
    "c2": (1_000_000, 100_000, 50_000_000, 64, 2),
    "small": (200_000, 50_000, 10_000_000, 128, 5),
    # C3's matrix at k = 256 (multi-wave row kernel)
    "c5": (10_000_000, 1_000_000, 500_000_000, 256, 3),
    # BPR: C2's matrix, k=64, 3 negatives, lr 0.05, no biases
    "c4": (1_000_000, 100_000, 50_000_000, 64, 2),
    # C3 with Zipf(1.0) item popularity: 550M draws -> ~502M unique pairs; ~2400 items hold
    # more than 16K signals (the largest ~9.4M), ~690K items at most 128
    "c3z": (10_000_000, 1_000_000, 550_000_000, 128, 3),
    # C5 with the same Zipf(1.0) item popularity: the split-K heavy rows at k = 256
    "c5z": (10_000_000, 1_000_000, 550_000_000, 256, 3),
    # the ML-100K-shaped synthetic (Appendix C, seed 1234; the committed
    # fixture tests/golden/ml100k_shape.npz), k = 30, 10 epochs = one step (bench_c1)
    "c1": (943, 1682, 100_000, 30, 1234),
}
ZIPF = {"c3z": 1.0, "c5z": 1.0}
BPR_CONFIGS = {"c4"}
C1_EPOCHS, C1_THREADS = 10, 4  # wals.cpp defaults for C1: 10 epochs, the CPU path at nthreads=4
LAM, ALPHA = 0.05, 40.0
PEAK_F32_TFLOPS = 157.3   # MI355X dense fp32 (MFMA = vector), MI355X_MICROARCH.md
PEAK_F64_TFLOPS = 78.6
PEAK_HBM_GBS = 8000.0
PEAK_ATOMIC_GBS = 1300.0  # chip-wide float atomic adds (MI355X_MICROARCH.md, measured)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


MKL = "/opt/conda/lib/libmkl_rt.so.1"


_CPU_SHARE = None


def cpu_share():
    """Threads for the CPU baseline: `nproc` (which honours OMP_NUM_THREADS, as the box sets
    it to its CPU share), bounded by the affinity mask and the cgroup CPU quota.  Taken once,
    before oracle_lib() sets OMP_NUM_THREADS=1 for the port."""
    global _CPU_SHARE
    if _CPU_SHARE is None:
        _CPU_SHARE = _cpu_share()
    return _CPU_SHARE


def _cpu_share():
    import subprocess
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = max(1, int(q) // int(per))
    except Exception:
        pass
    try:
        nproc = int(subprocess.run(["nproc"], capture_output=True, text=True).stdout.strip())
    except Exception:
        nproc = aff
    n = min(x for x in (nproc, aff, quota) if x)
    return n, {"nproc": nproc, "affinity": aff, "cgroup_cpu_quota": quota}


def oracle_lib():
    """The oracle with the host LAPACK's dsysv_ when the image has one (MKL, sequential: the
    survey's reference build, BASELINE.md CPU-baseline plan), else the restated netlib
    dsytf2/dsytrs.  Returns (pyoracle module, LAPACK description)."""
    if os.path.exists(MKL) and "ORC_LAPACK" not in os.environ:
        os.environ["ORC_LAPACK"] = MKL
        os.environ["MKL_THREADING_LAYER"] = "SEQUENTIAL"
        os.environ["MKL_NUM_THREADS"] = "1"
    os.environ["OMP_NUM_THREADS"] = "1"
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as po
    lap = os.environ.get("ORC_LAPACK")
    return po, ("dsysv_ from %s (sequential)" % lap) if lap else \
        "restated netlib dsytf2+dsytrs (no host LAPACK)"


def cpu_baseline(ctx, cfg, nthreads, budget_s=20.0):
    """Reference-structure CPU port (oracle/qmf_oracle.cpp: hash lookup per nnz, per-row
    k×k copies, full k×k Gram, dsysv, serial YᵀY) timed on a bounded sample of the SAME
    matrix: strided rows of each half and YᵀY over a row subset, scaled to one epoch."""
    po, lapack = oracle_lib()
    nu, ni, _, k, _ = cfg
    urp, ucol, uval = ctx.download_csr(0)
    irp, icol, ival = ctx.download_csr(1)
    U = ctx.factors(0)
    I = ctx.factors(1)
    total = 0.0
    detail = {"lapack": lapack}
    for side in (0, 1):
        rp, col, val = (urp, ucol, uval) if side == 0 else (irp, icol, ival)
        Y = I if side == 0 else U
        nL = nu if side == 0 else ni
        nR = ni if side == 0 else nu
        # sample rows: about budget/4 seconds of row solves per side
        avg_nnz = rp[-1] / nL
        est_row_s = (avg_nnz * k * k * 2.5e-10 + k ** 3 * 7e-11) / max(nthreads, 1)
        S = int(max(nthreads * 4, min(nL, budget_s / 4 / est_row_s)))
        rows = np.linspace(0, nL - 1, S).astype(np.int64)
        # compact sub-problem: sampled rows + the fixed-side rows they touch (+ a YtY sample)
        seg = [np.arange(rp[r], rp[r + 1]) for r in rows]
        idx = np.concatenate(seg)
        cols = col[idx]
        m_R = int(min(nR, max(20000, int(budget_s / 4 / (k * k * 1.0e-9)))))
        uniq = np.unique(np.concatenate([cols, np.arange(m_R)]))
        remap = np.searchsorted(uniq, cols).astype(np.int32)
        srp = np.concatenate([[0], np.cumsum([s.size for s in seg])]).astype(np.int64)
        dummy_rp = np.zeros(len(uniq) + 1, np.int64)
        args = (srp, remap, val[idx], dummy_rp,
                np.zeros(1, np.int32), np.zeros(1)) if side == 0 else \
               (dummy_rp, np.zeros(1, np.int32), np.zeros(1), srp, remap, val[idx])
        nsu, nsi = (S, len(uniq)) if side == 0 else (len(uniq), S)
        o = po.OracleWALS.from_csr(nsu, nsi, *args, k, LAM, ALPHA)
        o.set_factors(1 - side, Y[uniq])
        t_yty, t_rows, done = o.time_sample(side, nthreads, 1)
        # YtY in the sub-problem covered len(uniq) rows; the reference does all nR serially
        yty_full = t_yty * nR / len(uniq)
        rows_full = t_rows * nL / done
        detail["side%d" % side] = dict(rows_sampled=done, yty_rows=len(uniq),
                                       t_yty=t_yty, t_rows=t_rows)
        total += yty_full + rows_full
    return total, detail


def cpu_epoch(ctx, cfg, nthreads):
    """One FULL epoch of the reference-structure port (both halves, serial YᵀY, every row)
    on this matrix from the device's current item factors (the default baseline; minutes at
    C3, so main() runs it under a time guard)."""
    po, lapack = oracle_lib()
    nu, ni, _, k, _ = cfg
    t0 = time.perf_counter()
    urp, ucol, uval = ctx.download_csr(0)
    irp, icol, ival = ctx.download_csr(1)
    o = po.OracleWALS.from_csr(nu, ni, urp, ucol, uval, irp, icol, ival, k, LAM, ALPHA)
    del urp, ucol, uval, irp, icol, ival
    o.set_factors(1, ctx.factors(1))
    t_build = time.perf_counter() - t0
    log("cpu epoch: oracle built in %.1fs; running one epoch on %d threads" % (t_build, nthreads))
    import threading
    done = threading.Event()

    def heartbeat():  # the port runs minutes inside one ctypes call (GIL released)
        while not done.wait(30.0):
            log("cpu epoch: running, %.0fs" % (time.perf_counter() - t1))
    t1 = time.perf_counter()
    hb = threading.Thread(target=heartbeat, daemon=True)
    hb.start()
    o.iterate(0, nthreads)
    t_u = time.perf_counter() - t1
    log("cpu epoch: user half %.1fs" % t_u)
    loss = o.iterate(1, nthreads)
    t = time.perf_counter() - t1
    done.set()
    return t, {"lapack": lapack, "t_user_half": round(t_u, 3), "t_item_half": round(t - t_u, 3),
               "t_build": round(t_build, 3), "loss": loss}


def parity_check(ctx, cfg, nthreads, cfg_precision, nsample=1000, nheavy=16):
    """Full-size parity: one more (untimed) epoch; `nsample` rows of each half (plus its
    `nheavy` heaviest rows, reported apart) are re-solved
    by the oracle's updateFactorsForOne (WALSEngine.cpp:266-310) against the fixed side the
    device used (its own values), and compared with the device's rows and row losses."""
    po, _ = oracle_lib()
    nu, ni, _, k, seed = cfg
    rng = np.random.default_rng(seed + 7)
    I_prev = ctx.factors(1)
    ctx.wals_half(0, ALPHA, LAM)
    U, lu = ctx.factors(0), ctx.row_losses(0)
    ctx.wals_half(1, ALPHA, LAM)
    I, li = ctx.factors(1), ctx.row_losses(1)
    out = {"rows_per_half": nsample, "heaviest_rows_added": nheavy}
    worst = 0.0
    for side, Y, X, rl in ((0, I_prev, U, lu), (1, U, I, li)):
        rp, col, val = ctx.download_csr(side)
        nrow = len(rp) - 1
        # uniform sample + the `nheavy` heaviest rows (on skewed data the split-K heavy rows are
        # a few thousand of 1M: a uniform sample holds about 2 of them)
        heavy = np.argsort(np.diff(rp), kind="stable")[-nheavy:]
        uni = rng.choice(nrow, nsample, replace=False)
        rows = np.union1d(uni, heavy)
        t0 = time.perf_counter()
        x, loss = po.solve_rows(Y, rp, col, val, rows, ALPHA, LAM, nthreads)
        dev = X[rows]
        row_err = np.linalg.norm(dev - x, axis=1) / np.maximum(np.linalg.norm(x, axis=1), 1e-300)
        rel = float(np.linalg.norm(dev - x) / np.linalg.norm(x))
        lrel = float(np.max(np.abs(rl[rows] - loss) / np.maximum(np.abs(loss), 1e-300)))
        hv = np.isin(rows, heavy)
        out["side%d" % side] = {"max_row_rel_err": float(row_err.max()), "normwise_rel_err": rel,
                                "max_row_loss_rel_err": lrel,
                                "heavy_rows": int(hv.sum()),
                                "heavy_min_signals": int(np.diff(rp)[heavy].min()),
                                "heavy_max_row_rel_err": float(row_err[hv].max()),
                                "oracle_s": round(time.perf_counter() - t0, 2)}
        worst = max(worst, float(row_err.max()))
        del rp, col, val
    # the bar of the precision measured: fp64 is held to the GPU tests' 1e-9 (an fp64
    # regression between 1e-9 and 1e-4 must not print pass), fp32 to north_star's 1e-4
    tol = 1e-9 if cfg_precision == 64 else 1e-4
    out["max_rel_err"] = worst
    out["tolerance"] = tol
    out["pass"] = bool(worst <= tol)
    return out


# kernels of each timed class (names as rocprofv3 reports them)
CLASS_KERNELS = {
    "wals_direct_kernel": ("wals_direct_kernel<",),
    "wals_big_kernel": ("wals_big_kernel<",),
    "wals_whitened (row solve + unwhiten)": ("wals_woodbury_kernel<", "wals_woodbury_mw_kernel<",
                                             "wals_woodbury_st_kernel<", "wals_woodbury_st64_kernel<",
                                             "whiten_kernel<{T}, {NT}, true>"),
    "bpr_epoch_kernel": ("bpr_epoch_kernel<",),
}


def pmc_traffic(config, precision, cls, k):
    """HBM bytes per class launch from the newest committed PMC summary for this workload
    (profiles/rNN/pmc_<config>_<dtype>.json, written by tools/pmc_summary.py from
    rocprofv3 FETCH_SIZE/WRITE_SIZE passes; fetch already doubled per the gfx950 note)."""
    import glob
    dt = "f32" if precision == 32 else "f64"
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_%s_%s.json" % (config, dt))))
    if not files:
        return None, None
    ks = json.load(open(files[-1]))["kernels"]
    T = "float" if precision == 32 else "double"
    pats = [p.format(T=T, NT=(k + 15) // 16) for p in CLASS_KERNELS[cls]]
    tot, hit = 0.0, False
    for name, e in ks.items():
        if any(name.startswith(p) for p in pats) and "fetch_bytes" in e and "write_bytes" in e:
            # the largest dispatch = the class's large launch (older summaries: the mean)
            tot += e.get("fetch_bytes_max", e["fetch_bytes"]) + e.get("write_bytes_max", e["write_bytes"])
            hit = True
    return (tot if hit else None), os.path.relpath(files[-1], ROOT)


def eval_triplets(urp, ucol, ni, num_neg, seed):
    """Every positive × num_neg negatives rejected against the user's positives (the
    shape of BPREngine's evaluation set, BPREngine.cpp:85-87)."""
    rng = np.random.default_rng(seed)
    nu = len(urp) - 1
    users = np.repeat(np.arange(nu, dtype=np.int64), np.diff(urp))
    u = np.repeat(users, num_neg)
    p = np.repeat(ucol.astype(np.int64), num_neg)
    keys = users * ni + ucol  # CSR rows are sorted by column: keys ascending
    n = rng.integers(0, ni, len(u))
    for _ in range(64):
        q = u * ni + n
        pos = np.searchsorted(keys, q)
        bad = (pos < len(keys)) & (keys[np.minimum(pos, len(keys) - 1)] == q)
        if not bad.any():
            break
        n[bad] = rng.integers(0, ni, int(bad.sum()))
    return np.stack([u, p, n], 1)


def bench_bpr(args, rank, world):
    """C4: one step = one Hogwild epoch over every positive × 3 negatives (qmfx_bpr_epoch)
    plus the evaluation-set loss (qmfx_bpr_eval), as BPREngine::optimize does per epoch."""
    import qmf_amd
    nu, ni, nnz_req, k, seed = CONFIGS[args.config]
    num_neg, lr, lam = 3, 0.05, (1.0, 0.025, 0.0025)
    ctx = qmf_amd.Context(k, args.precision, device=int(os.environ.get("LOCAL_RANK", "0")))
    nnz = ctx.gen_synthetic(nu, ni, nnz_req, seed)
    urp, ucol, _ = ctx.download_csr(0)
    users = np.repeat(np.arange(nu, dtype=np.int64), np.diff(urp))
    # positives in a shuffled "file" order
    perm = np.random.default_rng(seed).permutation(nnz)
    ctx.bpr_set_positives(users[perm], ucol[perm].astype(np.int64))
    ctx.fill_uniform(0, 0.01, seed + 100)
    ctx.fill_uniform(1, 0.01, seed + 101)
    ctx.bpr_set_biases(np.zeros(ni))
    trip = eval_triplets(urp, ucol, ni, num_neg, seed)
    del users, perm
    ctx.sync()
    log("c4: data ready (%d positives, %d eval triplets)" % (nnz, len(trip)))

    def step(e):
        ctx.bpr_epoch(seed * 1000 + e, num_neg, lr * 0.9 ** e, *lam, False, shuffle=e > 0)
        return ctx.bpr_eval(0, trip, False) / len(trip)

    for e in range(args.warmup):
        step(e)
    ctx.reset_stats()
    ctx.sync()
    t1 = time.perf_counter()
    loss = 0.0
    for e in range(args.steps):
        loss = step(args.warmup + e)
    ctx.sync()
    el = time.perf_counter() - t1
    log("c4: %d timed epochs in %.3fs" % (args.steps, el))
    st = ctx.solve_stats()
    upd = nnz * num_neg * args.steps
    sec = st["ms"] / 1e3 / max(st["launches"], 1)
    by = st["bytes"] / max(st["launches"], 1)
    kp = (k + 15) // 16 * 16
    esz = 4 if args.precision == 32 else 8
    atomic_by = float(nnz) * (num_neg + 1) * kp * esz
    out = {
        "metric": "BPR Hogwild updates/sec at k=%d (epoch + evaluation pass)" % k,
        "value": round(upd / el, 1), "unit": "updates/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "replicas", "vs_baseline": None,
        "dtype": "f32" if args.precision == 32 else "f64",
        "data": "synthetic (device-generated uniform unique pairs, seed %d)" % seed,
        "config": {"workload": "%s: BPR %d users x %d items, %d positives x %d negatives, k=%d"
                   % (args.config, nu, ni, nnz, num_neg, k)},
        # The epoch is bound by the chip-wide float-atomic rate (MI355X_MICROARCH.md "Global
        # float atomics": ≈1.3 TB/s of added bytes): per positive the item rows q_p and the
        # num_neg q_n are added atomically (the user row is a plain store); the HBM fraction of
        # the algorithmic bytes (≈1.6 KB per update) is reported beside it
        "roofline": {"kernel": "bpr_epoch_kernel", "bound": "l2_atomic",
                     "achieved": round(atomic_by / sec / 1e9, 1), "peak": PEAK_ATOMIC_GBS,
                     "unit": "GB/s", "frac": round(atomic_by / sec / 1e9 / PEAK_ATOMIC_GBS, 4),
                     "atomic_bytes_per_launch": atomic_by,
                     "hbm": {"achieved": round(by / sec / 1e9, 1), "peak": PEAK_HBM_GBS,
                             "frac": round(by / sec / 1e9 / PEAK_HBM_GBS, 4),
                             "bytes_per_launch": by},
                     "launch_ms": round(sec * 1e3, 3)},
        "eval_loss": loss,
        "env": engine_env(os.environ),
    }
    variant = qmf_amd._abi.build_variant()
    if variant:
        out["variant"] = variant
    traffic, tsrc = pmc_traffic(args.config, args.precision, "bpr_epoch_kernel", k)
    out["roofline"].update({"traffic": round(traffic, 0) if traffic else None,
                            "traffic_algorithmic_ratio": round(traffic / by, 3) if traffic else None,
                            "traffic_source": tsrc})
    if args.cpu_baseline != "none" and rank == 0:
        # one full reference-structure Hogwild epoch (BPREngine::optimize with
        # numHogwildThreads = nthreads) + its evaluation pass, from the device's factors, at
        # the learning rate the NEXT epoch uses (lr·decay^epochs, BPREngine.cpp:169-171); the
        # device runs that same next epoch from the same state, so both eval losses are
        # like for like (round 2 gave the port the undecayed lr: 0.05 late in training makes
        # the item factors grow and the loss rise, 0.56 → 2.44)
        po, _ = oracle_lib()
        nthreads, host = cpu_share()
        e_next = args.warmup + args.steps
        lr_next = lr * 0.9 ** e_next
        log("c4: CPU baseline (one Hogwild epoch, %d threads, lr %.4g)" % (nthreads, lr_next))
        U, I = ctx.factors(0), ctx.factors(1)
        b = np.zeros(ni)
        users = np.repeat(np.arange(nu, dtype=np.int64), np.diff(urp))
        perm = np.random.default_rng(seed).permutation(nnz)
        t_up, t_ev, closs = po.bpr_hogwild_epoch(U, I, b, users[perm], ucol[perm], ni, num_neg,
                                                 nthreads, seed, lr_next, *lam, False, trip)
        dloss = step(e_next)  # the device's same next epoch (untimed)
        t = t_up + t_ev
        out["cpu_baseline"] = {"value": round(nnz * num_neg / t, 1), "unit": "updates/s",
                               "cores": nthreads, "kind": "port", "ms_per_epoch": round(t * 1e3, 1),
                               "sample": "one full Hogwild epoch (%d threads, %d updates) + the "
                                         "evaluation pass of the reference-structure port on "
                                         "this workload: %.1f s + %.1f s" % (nthreads, nnz * num_neg,
                                                                             t_up, t_ev),
                               "detail": {"host": host, "lr": lr_next,
                                          "eval_loss": closs / len(trip),
                                          "device_eval_loss_same_epoch": dloss}}
    if rank == 0 and not args.no_parity:
        # the update rule, exact: a sample of triplets (positives with their negatives) applied
        # in sequence by qmfx_bpr_apply and by the oracle's BPREngine::update restatement
        # (BPREngine.cpp:178-220) from the same factors (Hogwild epochs are statistical; SURVEY
        # §0.7)
        po, _ = oracle_lib()
        rng = np.random.default_rng(seed + 9)
        ns = 20000
        sample = trip[rng.choice(len(trip), ns, replace=False)]
        U0, I0 = ctx.factors(0), ctx.factors(1)
        b0 = np.zeros(ni)
        lr_s = lr * 0.9 ** (args.warmup + args.steps)
        ctx.bpr_set_biases(b0)
        ctx.bpr_apply(sample, lr_s, *lam, False)
        U, I = U0.copy(), I0.copy()
        po.bpr_update_seq(U, I, b0.copy(), sample, lr_s, *lam, False)
        err = max(float(np.max(np.abs(ctx.factors(0) - U)) / np.max(np.abs(U))),
                  float(np.max(np.abs(ctx.factors(1) - I)) / np.max(np.abs(I))))
        tol = 1e-12 if args.precision == 64 else 1e-5
        out["parity"] = {"check": "qmfx_bpr_apply vs the oracle's BPREngine::update, %d sampled "
                                  "triplets in sequence from the device's factors" % ns,
                         "max_rel_err": err, "tolerance": tol, "pass": bool(err <= tol)}
        del U0, I0, U, I
    if rank == 0:
        print(json.dumps(out), flush=True)


def class_stats(ctx):
    """The context's kernel-class accounting: {class name: {"total": stats, "side": {side:
    stats}}} with stats = dict(ms, launches, flops, bytes) (qmfx_kernel_stats[_side])."""
    out = {}
    for cls, name in ((0, "direct"), (1, "whitened")):
        out[name] = {"total": ctx.kernel_stats(cls),
                     "side": {sd: ctx.kernel_stats_side(cls, sd) for sd in (0, 1)}}
    return out


def bench_c1(args, rank):
    """C1 (BASELINE configs[0]): the reference's CPU-runnable case, `wals` on the ML-100K shape
    (943 × 1682, 100K signals, Appendix C generator, seed 1234), k = 30, λ 0.05, α 40, the item
    factors from the seeded distribution file, 10 epochs.  One step = the whole 10-epoch run
    from the same initial factors (qmf/wals.cpp:52-107: set factors, optimize).  The ingest
    (device grouping of the triples) is done once, before the timed steps.  cpu_baseline: the
    reference-structure port, the same 10 epochs at nthreads = 4 (the config's definition);
    parity: the device's per-epoch losses and final factors against the port's, and its
    epoch-1 / epoch-10 losses against the reference's printed values."""
    import qmf_amd
    d = np.load(os.path.join(ROOT, "tests", "golden", "ml100k_shape.npz"))
    users, items = d["users"].astype(np.int64), d["items"].astype(np.int64)
    values = d["values"].astype(np.float64)
    init = d["init_e9"].astype(np.float64) / 1e9
    nu0, ni0, nnz0, k, seed = CONFIGS["c1"]
    ctx = qmf_amd.Context(k, args.precision, device=int(os.environ.get("LOCAL_RANK", "0")))
    ctx.group_signals(users, items, values)
    nu, ni = ctx.nusers, ctx.nitems
    assert (nu, ni, len(users)) == (nu0, ni0, nnz0), (nu, ni, len(users))
    I0 = init[: ni * k].reshape(ni, k)

    def run():
        ctx.set_factors(1, I0)
        out = []
        for _ in range(C1_EPOCHS):
            ctx.wals_half(0, ALPHA, LAM)
            out.append(ctx.wals_half(1, ALPHA, LAM) / nu / ni)
        return out

    for _ in range(args.warmup):
        run()
    ctx.reset_stats()
    ctx.sync()
    t1 = time.perf_counter()
    losses = None
    for _ in range(args.steps):
        losses = run()
    ctx.sync()
    el = time.perf_counter() - t1
    solves = (nu + ni) * C1_EPOCHS * args.steps
    classes = roofline_classes(class_stats(ctx), k, args.precision,
                               {sd: int(sum(ctx.row_classes(sd)["whitened"])) for sd in (0, 1)})
    roof = roofline_object(classes)
    roof["classes"] = classes
    out = {
        "metric": "WALS solves/sec and ms/epoch at k=%d; achieved fraction of HBM roofline" % k,
        "value": round(solves / el, 1), "unit": "solves/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3),
        "ms_per_epoch": round(el / args.steps / C1_EPOCHS * 1e3, 3),
        "higher_is_better": True, "scaling": "replicas", "vs_baseline": None,
        "dtype": "f32" if args.precision == 32 else "f64",
        "data": "synthetic ML-100K shape (SURVEY.md Appendix C generator, seed 1234; "
                "tests/golden/ml100k_shape.npz), item factors from the seeded distribution file",
        "config": {"workload": "c1: %d users x %d items, %d nnz, k=%d, lambda=%g, alpha=%g, "
                               "%d epochs per step" % (nu, ni, len(users), k, LAM, ALPHA, C1_EPOCHS),
                   "nusers": nu, "nitems": ni, "nnz": len(users), "nfactors": k,
                   "epochs_per_step": C1_EPOCHS, "parallelism": "rows1"},
        "roofline": roof, "loss": losses[-1], "env": engine_env(os.environ),
    }
    variant = qmf_amd._abi.build_variant()
    if variant:
        out["variant"] = variant
    if rank == 0 and (args.cpu_baseline != "none" or not args.no_parity):
        po, lapack = oracle_lib()
        o = po.OracleWALS(users, items, values, k, LAM, ALPHA)
        o.set_factors(1, I0)
        t0 = time.perf_counter()
        closs = o.optimize(C1_EPOCHS, C1_THREADS)
        tcpu = time.perf_counter() - t0
        if args.cpu_baseline != "none":
            out["cpu_baseline"] = {
                "value": round((nu + ni) * C1_EPOCHS / tcpu, 1), "unit": "solves/s",
                "cores": C1_THREADS, "kind": "port", "ms_per_step": round(tcpu * 1e3, 1),
                "sample": "the whole C1 run (10 epochs, nthreads=4, the config's definition) of the "
                          "reference-structure port: %.2f s" % tcpu,
                "detail": {"lapack": lapack, "host": cpu_share()[1]}}
        if not args.no_parity:
            err = max(float(np.max(np.abs(ctx.factors(sd) - o.factors(sd))) /
                            np.max(np.abs(o.factors(sd)))) for sd in (0, 1))
            lerr = max(abs(a - b) / abs(b) for a, b in zip(losses, closs))
            ref = (float(d["ref_loss_epoch1"]), float(d["ref_loss_epoch10"]))
            # after 10 epochs (tests/test_cli_gpu.py's bar): fp64 1e-8, fp32 north_star's 1e-4;
            # the reference prints its losses to 6 significant digits
            tol = 1e-8 if args.precision == 64 else 1e-4
            out["parity"] = {
                "max_factor_rel_err_vs_port": err, "max_epoch_loss_rel_err_vs_port": lerr,
                "loss_epoch1": losses[0], "loss_epoch10": losses[-1],
                "reference_printed_losses": ref, "tolerance": tol,
                "pass": bool(err <= tol and abs(losses[0] - ref[0]) < 1e-5
                             and abs(losses[-1] - ref[1]) < 1e-6)}
    if rank == 0:
        print(json.dumps(out), flush=True)


def roofline_classes(stats, k, precision, whitened_rows=None):
    """Per kernel class and side: the launch's algorithmic flops and bytes (the
    class's rows' signals, gathered rows, X writes and rowptr; the YᵀY read runs in its own
    kernel) over its HIP-event time, the bound (MFMA when the launch's intensity is above the
    ridge, else HBM) and the fraction of that peak.  A class's top-level fields are its LARGE
    launch's (the side whose launches take longest: the C3 direct kernel runs 187 ms in the item
    half and 69 us in the user half); `per_side` has both.  whitened_rows[side]: the side's
    n×n-route rows, whose x' round trip (written after the solve, read by the unwhitening pass:
    2·k·s per row) is reported as `extra_bytes` beside the §8(d) bytes, not inside them."""
    peak_tf = PEAK_F32_TFLOPS if precision == 32 else PEAK_F64_TFLOPS
    ridge = peak_tf * 1e12 / (PEAK_HBM_GBS * 1e9)
    esz = 4 if precision == 32 else 8
    names = {"direct": "wals_big_kernel" if k > 128 else "wals_direct_kernel",
             "whitened": "wals_whitened (row solve + unwhiten)"}
    classes = {}
    for cls, name in names.items():
        tot = stats[cls]["total"]
        if tot["launches"] == 0 or tot["ms"] <= 0:
            continue
        per = {}
        for side in (0, 1):
            st = stats[cls]["side"][side]
            if not (st["launches"] and st["ms"] > 0):
                continue
            n = st["launches"]
            ms, fl, by = st["ms"] / n, st["flops"] / n, st["bytes"] / n
            sec = ms / 1e3
            tf, gbs = fl / sec / 1e12, by / sec / 1e9
            if fl / by >= ridge:
                bound, ach, pk, unit = "mfma", tf, peak_tf, "TFLOP/s"
            else:
                bound, ach, pk, unit = "hbm", gbs, PEAK_HBM_GBS, "GB/s"
            per[side] = dict(launch_ms=round(ms, 3), bound=bound, achieved=round(ach, 3), peak=pk,
                             unit=unit, frac=round(ach / pk, 4), tflops=round(tf, 3),
                             gbs=round(gbs, 1), flops_per_launch=fl, bytes_per_launch=by)
            if cls == "whitened" and whitened_rows is not None:
                per[side]["extra_bytes"] = float(2 * whitened_rows[side] * k * esz)
        side = max(per, key=lambda sd: per[sd]["launch_ms"])
        classes[name] = dict(per[side], side=side, total_ms=round(tot["ms"], 3),
                             launches=tot["launches"], per_side=per,
                             per_side_launch_ms={sd: v["launch_ms"] for sd, v in per.items()})
    return classes


# the line's headline class: the one with the most kernel time, except that within this margin
# the item half's class is named (C3 fp64's two classes tie within 0.1%: the headline flipped
# between runs in round 5)
HEADLINE_TIE = 0.05
ROOF_KEYS = ("bound", "achieved", "peak", "unit", "frac", "launch_ms", "bytes_per_launch",
             "flops_per_launch")


def roofline_object(classes):
    """The line's `roofline`: the headline class's fields, the weakest class, and both halves
    as fixed fields (`user_half`, `item_half`: the class with the longer launch on that side,
    with that side's launch figures)."""
    order = sorted(classes, key=lambda n: classes[n]["total_ms"], reverse=True)
    dom = order[0]
    if len(order) > 1 and classes[order[1]]["total_ms"] >= (1 - HEADLINE_TIE) * classes[dom]["total_ms"]:
        items = [n for n in order[:2] if classes[n]["side"] == 1]
        if items:
            dom = items[0]
    weak = min(classes, key=lambda n: classes[n]["frac"])
    d = classes[dom]
    roof = {"kernel": dom, **{k: d[k] for k in ROOF_KEYS}, "launch_side": d["side"],
            "weakest": {"kernel": weak, "bound": classes[weak]["bound"],
                        "frac": classes[weak]["frac"], "launch_ms": classes[weak]["launch_ms"]}}
    if "extra_bytes" in d:
        roof["extra_bytes"] = d["extra_bytes"]
    for side, field in ((0, "user_half"), (1, "item_half")):
        on = [n for n in classes if side in classes[n]["per_side"]]
        if on:
            best = max(on, key=lambda n: classes[n]["per_side"][side]["launch_ms"])
            ps = classes[best]["per_side"][side]
            roof[field] = {"kernel": best, **{k: ps[k] for k in ROOF_KEYS}}
            if "extra_bytes" in ps:
                roof[field]["extra_bytes"] = ps["extra_bytes"]
    return roof


T_START = time.time()
# seconds of the whole bench process the guarded CPU epoch may run into (the driver's limit
# is 600 s; the GPU part, the parity check and the sampled fallback come first)
TIME_LIMIT_S = float(os.environ.get("QMFX_BENCH_LIMIT_S", "540"))

# reference-structure port, one thread, measured in the survey container (SURVEY.md
# Appendix B): Gram per signal and dsysv_ per row, µs, by k
_GRAM_US = {30: 0.146, 64: 0.591, 128: 2.285, 256: 9.212}
_SOLVE_US = {30: 4.3, 64: 13.57, 128: 158.45, 256: 1407.3}


def cpu_epoch_estimate_s(nu, ni, nnz, k, nthreads):
    """Conservative wall-time model of one port epoch (both halves' rows over `nthreads`, the
    serial YᵀY at ≈1 ns per FMA): C3 on 16 threads → 431 s (measured 355.5 s)."""
    kk = min(_GRAM_US, key=lambda x: abs(x - k))
    g = _GRAM_US[kk] * (k / kk) ** 2
    sv = _SOLVE_US[kk] * (k / kk) ** 3
    rows = (2 * nnz * g + (nu + ni) * sv) * 1e-6 / max(nthreads, 1)
    return rows + (nu + ni) * k * k * 1e-9


def launch_plan(gpus, env, argv, port=None):
    """None when this process is a rank (or the run is single-GPU); otherwise the child
    command that runs `gpus` ranks under torch.distributed.run (one rank per GPU)."""
    if gpus <= 1 or "WORLD_SIZE" in env:
        return None
    if port is None:
        import socket
        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            port = so.getsockname()[1]
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            "--nproc-per-node=%d" % gpus, "--master-addr", "127.0.0.1",
            "--master-port=%d" % port, os.path.abspath(__file__)] + list(argv)


def check_world(gpus, world, visible=None, local=0):
    """Raises SystemExit unless the launcher started exactly `gpus` ranks and this rank's
    GPU exists."""
    if world != gpus:
        raise SystemExit("bench.py: --gpus %d but the launcher started %d rank(s)" % (gpus, world))
    if visible is not None and local >= visible:
        raise SystemExit("bench.py: --gpus %d needs %d GPUs; rank %d sees only %d"
                         % (gpus, gpus, local, visible))


# QMFX_* variables that make a run skip work (timing experiments): a line measured under one
# is not a measurement of the product, so the bench refuses to print it
WORK_SKIPPING_ENV = ("QMFX_ABLATE",)
# variables of the harness itself (not engine knobs)
_HARNESS_ENV = ("QMFX_BENCH_LIMIT_S",)


def engine_env(environ):
    """The QMFX_* engine knobs set in this run's environment (all are reported in the line)."""
    return {k: v for k, v in sorted(environ.items())
            if k.startswith("QMFX_") and k not in _HARNESS_ENV}


def check_env(environ, variant, allow_variant=False):
    """Raises SystemExit when the run would not measure the product: a work-skipping knob is
    set, or the loaded library is a timing-variant build (qmfx_build_variant() != "") and
    --allow-variant was not given."""
    bad = [k for k in WORK_SKIPPING_ENV if environ.get(k, "0") not in ("", "0")]
    if bad:
        raise SystemExit("bench.py: %s set: the run would skip work; refusing to report a line"
                         % ", ".join(bad))
    if variant and not allow_variant:
        raise SystemExit("bench.py: the loaded library is a timing-variant build (%s); "
                         "pass --allow-variant to measure it anyway (the line is marked)" % variant)


# the exchange model of DESIGN.md §6: a rank receives (W − 1)/W of the solved side's factor
# matrix per half; "bus" is the all-gather bus rate RCCL reaches on 8-GPU MI300-class nodes
# (an assumption the first SCALE run tests), "links" the receive bound of a fully connected
# 8-GPU xGMI mesh (7 links × 153 GB/s)
MODEL_BUS_GBS, MODEL_LINKS_GBS = 350.0, 1071.0


def exchange_model(nrows, kp, esz, world):
    """Predicted per-half exchange: bytes received per rank and their time at the model rates."""
    b = nrows * kp * esz * (world - 1) / world
    return {"bytes_in_per_rank": float(b), "model_ms_bus": round(b / MODEL_BUS_GBS / 1e6, 3),
            "model_ms_links": round(b / MODEL_LINKS_GBS / 1e6, 3)}


def exchange_fields(stats, steps, reduce_max, model=None):
    """Per half (users, items) of a multi-rank run: the exchange on the collective stream and
    the row solves, ms per half, each the max over ranks (reduce_max: list of floats -> the
    elementwise max over ranks).  stats[side] = Context.exchange_stats(side) (sums over the
    timed halves); model[side] = exchange_model(...) of that half, printed beside the measured
    exchange so the first multi-GPU record tests DESIGN.md §6 directly."""
    keys = ("exchange_ms", "exposed_ms", "solve_ms")
    vals = [stats[side][k] / max(steps, 1) for side in (0, 1) for k in keys]
    vals = reduce_max(vals)
    out = {}
    for side, name in ((0, "user_half"), (1, "item_half")):
        out[name] = {k: round(vals[3 * side + i], 3) for i, k in enumerate(keys)}
        if model is not None:
            out[name]["predicted"] = model[side]
            bus = model[side]["bytes_in_per_rank"] / max(out[name]["exchange_ms"], 1e-9) / 1e6
            out[name]["measured_gbs_in_per_rank"] = round(bus, 1)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--precision", type=int, default=64, choices=(32, 64))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-baseline", default="epoch", choices=("sample", "epoch", "none"))
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--allow-variant", action="store_true",
                    help="measure a timing-variant library (QMFX_LIB); the line is marked")
    args = ap.parse_args()
    if args.no_cpu_baseline:
        args.cpu_baseline = "none"
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")

    # N ranks: relaunch under torch.distributed.run as a CHILD process before anything
    # touches the GPU (this process never initialises HIP), and exit with its status
    cmd = launch_plan(args.gpus, os.environ, sys.argv[1:])
    if cmd is not None:
        log("bench.py: launching %d ranks: %s" % (args.gpus, " ".join(cmd)))
        import subprocess
        sys.exit(subprocess.run(cmd).returncode)

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    check_world(args.gpus, world)

    import qmf_amd

    variant = qmf_amd._abi.build_variant()
    check_env(os.environ, variant, args.allow_variant)
    check_world(args.gpus, world, qmf_amd.device_count(), local)
    cpu_share()
    if args.config == "c1":
        return bench_c1(args, rank)
    if args.config in BPR_CONFIGS:
        # BPR shards nothing (Hogwild across GPUs would need cross-device atomics): every
        # rank runs an independent replica; rank 0 reports
        return bench_bpr(args, rank, 1)

    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
    nu, ni, nnz_req, k, seed = CONFIGS[args.config]
    zipf = ZIPF.get(args.config, 0.0)

    t0 = time.time()
    ctx = qmf_amd.Context(k, args.precision, device=local)
    if zipf:
        nnz = ctx.gen_synthetic_zipf(nu, ni, nnz_req, seed, zipf)
    else:
        nnz = ctx.gen_synthetic(nu, ni, nnz_req, seed)
    ctx.fill_uniform(1, 0.01, seed + 100)
    if world > 1:
        uid = [qmf_amd.rccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        ctx.dist_init(rank, world, uid[0])
    ctx.sync()
    log("rank %d: data ready in %.1fs (nnz=%d)" % (rank, time.time() - t0, nnz))

    def epoch():
        ctx.wals_half(0, ALPHA, LAM)
        return ctx.wals_half(1, ALPHA, LAM)

    for _ in range(args.warmup):
        epoch()
    ctx.reset_stats()
    if dist:
        dist.barrier()
    ctx.sync()
    t1 = time.perf_counter()
    loss = 0.0
    for _ in range(args.steps):
        loss = epoch()
    ctx.sync()
    el = time.perf_counter() - t1
    if dist:
        import torch
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t[0])
        dist.barrier()
    ms_epoch = el / args.steps * 1e3
    solves = (nu + ni) * args.steps
    value = solves / el
    wrows = {}
    for sd in (0, 1):
        wrows[sd] = int(sum(ctx.row_classes(sd)["whitened"]))  # this rank's n×n-route rows
    classes = roofline_classes(class_stats(ctx), k, args.precision, wrows)
    # the headline class (roofline_object) carries the line's roofline; the class furthest
    # below its own roofline and both halves' classes are named beside it
    roof = roofline_object(classes)
    dom = roof["kernel"]
    d = classes[dom]
    # PMC bytes of the same (large) launch, from the newest committed summary for this workload
    traffic, tsrc = pmc_traffic(args.config, args.precision, dom, k)
    roof.update({"traffic": round(traffic, 0) if traffic else None,
                 "traffic_algorithmic_ratio": round(traffic / d["bytes_per_launch"], 3) if traffic else None,
                 # the counted L2<->fabric bytes per launch over this run's launch time (MALL hits
                 # included: the fabric rate the class runs at)
                 "traffic_gbs": round(traffic / (d["launch_ms"] / 1e3) / 1e9, 1) if traffic else None,
                 "traffic_source": tsrc, "classes": classes})
    xfields = None
    if dist:
        # the exchange per half, each field the max over ranks
        def reduce_max(vals):
            import torch
            t = torch.tensor(vals, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return [float(v) for v in t]
        kp = (k + 15) // 16 * 16
        esz = 4 if args.precision == 32 else 8
        model = {0: exchange_model(nu, kp, esz, world), 1: exchange_model(ni, kp, esz, world)}
        xfields = exchange_fields({sd: ctx.exchange_stats(sd) for sd in (0, 1)}, args.steps,
                                  reduce_max, model)
    half = ctx.kernel_stats(2)
    epoch_bytes = half["bytes"] / max(half["launches"], 1) * 2
    hbm_frac_epoch = epoch_bytes / (ms_epoch / 1e3) / (PEAK_HBM_GBS * 1e9)
    if rank != 0:
        return
    out = {
        "metric": "WALS solves/sec and ms/epoch at k=%d; achieved fraction of HBM roofline" % k,
        "value": round(value, 1),
        "unit": "solves/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_epoch, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32" if args.precision == 32 else "f64",
        "data": ("synthetic (device-generated: uniform users, Zipf(%g) item popularity, w in "
                 "1..5, seed %d)" % (zipf, seed)) if zipf else
                "synthetic (device-generated uniform unique pairs, w in 1..5, seed %d)" % seed,
        "config": {"workload": "%s: %d users x %d items, %d nnz, k=%d, lambda=%g, alpha=%g"
                   % (args.config, nu, ni, nnz, k, LAM, ALPHA),
                   "nusers": nu, "nitems": ni, "nnz": nnz, "nfactors": k,
                   "parallelism": "rows%d" % world},
        "roofline": roof,
        "hbm_roofline_frac_epoch": round(hbm_frac_epoch, 4),
        "loss": loss / nu / ni,
        "env": engine_env(os.environ),
    }
    if variant:
        out["variant"] = variant
    if xfields is not None:
        out["exchange"] = xfields
    nthreads, host = cpu_share()
    if not args.no_parity and world == 1:
        t0 = time.perf_counter()
        out["parity"] = parity_check(ctx, CONFIGS[args.config], nthreads, args.precision)
        log("parity check %.1fs: %s" % (time.perf_counter() - t0, out["parity"]))
    if args.cpu_baseline != "none" and world == 1:
        cfg = (nu, ni, nnz, k, seed)

        def baseline(tcpu, sample, detail):
            detail["host"] = host
            return {"value": round((nu + ni) / tcpu, 1), "unit": "solves/s", "cores": nthreads,
                    "kind": "port", "ms_per_epoch": round(tcpu * 1e3, 1), "sample": sample,
                    "detail": detail}

        def sampled(budget):
            tcpu, detail = cpu_baseline(ctx, CONFIGS[args.config], nthreads, budget)
            return baseline(tcpu, "strided row samples of each half of this matrix and YtY on "
                                  "a row subset, scaled to one epoch = %.1f s" % tcpu, detail)

        if args.cpu_baseline == "epoch":
            est = cpu_epoch_estimate_s(nu, ni, nnz, k, nthreads)
            left = TIME_LIMIT_S - (time.time() - T_START)
            log("cpu baseline: one full epoch, estimated %.0f s on %d threads; %.0f s left of "
                "the %.0f s time guard" % (est, nthreads, left, TIME_LIMIT_S))
            if est > left - 30:
                out["cpu_baseline"] = sampled(args.cpu_budget)
                out["cpu_baseline"]["sample"] += (" (the time guard skipped the full epoch: "
                                                  "estimated %.0f s, %.0f s left)" % (est, left))
            else:
                # fallback first, so the guard below always has a baseline to report
                fb = sampled(min(args.cpu_budget, 10.0))
                fb["sample"] += " (the time guard stopped the full epoch)"
                out["cpu_baseline"] = fb
                import threading

                def guard():  # the port runs minutes inside one ctypes call (GIL released)
                    rest = TIME_LIMIT_S - (time.time() - T_START)
                    if not finished.wait(max(rest, 1.0)):
                        log("cpu baseline: time guard hit, reporting the sampled estimate")
                        print(json.dumps(out), flush=True)
                        os._exit(0)
                finished = threading.Event()
                threading.Thread(target=guard, daemon=True).start()
                tcpu, detail = cpu_epoch(ctx, cfg, nthreads)
                finished.set()
                detail["sampled_estimate_s"] = round(fb["ms_per_epoch"] / 1e3, 1)
                out["cpu_baseline"] = baseline(
                    tcpu, "one full epoch (user half + item half, every row, serial YtY) of "
                          "the reference-structure port on this matrix: %.1f s" % tcpu, detail)
        else:
            out["cpu_baseline"] = sampled(args.cpu_budget)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
