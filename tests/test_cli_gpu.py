"""End-to-end parity of the drop-in CLIs on the MI355X: `wals` / `bpr` (qmf_amd/bin) run
with the reference's flags, their output files (Engine::saveFactors text) and log lines
compared with the oracle run on the same inputs.

Tolerances: fp64 (the default) 1e-8 normwise-relative on factors (the files round to 9
decimals, so absolute 5e-10 per entry is the floor); fp32 1e-4 at the reference's λ/α on
well-posed inputs (10 epochs of the ML-100K shape included)."""
import os
import re
import subprocess

import numpy as np
import pytest

import pyoracle as po
from helpers import ROOT, load_ml100k, load_tiny, rel_err, synth

pytestmark = pytest.mark.gpu
BIN = os.path.join(ROOT, "qmf_amd", "bin")


def run(exe, *flags, timeout=300):
    r = subprocess.run([os.path.join(BIN, exe)] + list(flags), capture_output=True, text=True,
                       timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    return r.stderr


def read_factors(path, biases=False):
    rows = [line.split(" ") for line in open(path).read().splitlines()]
    ids = np.array([int(r[0]) for r in rows], np.int64)
    vals = np.array([[float(x) for x in r[1:]] for r in rows])
    if biases:
        return ids, vals[:, 0], vals[:, 1:]
    return ids, vals


def write_dataset(path, users, items, values):
    with open(path, "w") as f:
        for u, i, v in zip(users, items, values):
            f.write("%d %d %r\n" % (u, i, float(v)))


def write_dist(path, init):
    with open(path, "w") as f:
        f.write("".join("%.9f\n" % x for x in np.ravel(init)))


# the log prints losses with ostream's default 6 significant digits, as the reference
LOG_RTOL = 5e-6


def losses(log):
    return [float(x) for x in re.findall(r"epoch \d+: train loss = ([-\d.e+]+)", log)]


def wals_vs_oracle(tmp_path, users, items, values, k, nepochs, precision, lam=0.05, alpha=40.0,
                   init=None, extra=()):
    data = str(tmp_path / "train.txt")
    write_dataset(data, users, items, values)
    o = po.OracleWALS(users, items, values, k, lam, alpha)
    if init is None:
        init = np.random.default_rng(k).uniform(-0.01, 0.01, (o.nitems, k))
    dist = str(tmp_path / "dist.dat")
    write_dist(dist, init)
    o.load_distribution_file(dist)
    uf, itf = str(tmp_path / "U.txt"), str(tmp_path / "I.txt")
    log = run("wals", "--train_dataset=" + data, "--nfactors=%d" % k, "--nepochs=%d" % nepochs,
              "--regularization_lambda=%r" % lam, "--confidence_weight=%r" % alpha,
              "--distribution_file=" + dist, "--user_factors=" + uf, "--item_factors=" + itf,
              *(("--precision=%d" % precision,) if precision else ()), *extra)
    ol = o.optimize(nepochs)
    ui, U = read_factors(uf)
    ii, I = read_factors(itf)
    assert np.array_equal(ui, o.ids(0)) and np.array_equal(ii, o.ids(1))
    return log, ol, U, I, o


def test_wals_cli_tiny_default_precision(tmp_path):
    """No --precision flag: the CLI computes in fp64 like the reference (Types.h:24), so the
    ill-conditioned edge-case fixture (9 users) matches the oracle to 1e-8."""
    u, i, v = load_tiny()
    log, ol, U, I, o = wals_vs_oracle(tmp_path, u, i, v, 8, 3, None)
    assert rel_err(U, o.factors(0)) < 1e-8 and rel_err(I, o.factors(1)) < 1e-8
    np.testing.assert_allclose(losses(log), ol, rtol=LOG_RTOL)


def test_wals_cli_fp32_well_posed(tmp_path):
    """--precision=32 at the reference's λ/α on a well-posed dataset: within 1e-4."""
    u, i, v = synth(3000, 800, 60000, seed=12)
    log, ol, U, I, o = wals_vs_oracle(tmp_path, u, i, v, 24, 3, 32)
    assert rel_err(U, o.factors(0)) < 1e-4 and rel_err(I, o.factors(1)) < 1e-4
    np.testing.assert_allclose(losses(log), ol, rtol=1e-4)


@pytest.mark.parametrize("precision,tol", [(64, 1e-8), (32, 1e-4)])
def test_wals_cli_ml100k_shape_matches_reference_losses(tmp_path, precision, tol):
    d = load_ml100k()
    k = 30
    init = d["init"][: 1682 * k].reshape(1682, k)
    log, ol, U, I, o = wals_vs_oracle(tmp_path, d["users"], d["items"], d["values"], k, 10,
                                      precision, init=init)
    ls = losses(log)
    assert len(ls) == 10
    # the reference's own printed losses, at 6 significant digits
    assert abs(ls[0] - float(d["ref_loss_epoch1"])) < 1e-5
    assert abs(ls[9] - float(d["ref_loss_epoch10"])) < 1e-6
    assert rel_err(U, o.factors(0)) < tol and rel_err(I, o.factors(1)) < tol


def test_wals_cli_indefinite_rows_are_resolved(tmp_path):
    # 1 + α·v < 0 with O(1) factors makes some user systems indefinite: the device flags
    # them and re-solves them in fp64 with a pivoted solve, where the reference's dsysv
    # would run Bunch-Kaufman.  One user half + one item half.
    u, i, v = synth(300, 80, 3000, seed=9)
    v = v.copy()
    v[::11] = -5.0
    init = np.random.default_rng(1).uniform(0.2, 0.4, (80, 8))
    log, ol, U, I, o = wals_vs_oracle(tmp_path, u, i, v, 8, 1, 64, lam=0.01, init=init)
    assert "not positive definite; re-solved with pivoting" in log
    assert rel_err(U, o.factors(0)) < 1e-7 and rel_err(I, o.factors(1)) < 1e-7
    np.testing.assert_allclose(losses(log), ol, rtol=LOG_RTOL)


def test_wals_cli_test_metrics(tmp_path):
    u, i, v = synth(400, 150, 6000, seed=3)
    te = synth(400, 150, 1500, seed=30)
    test = str(tmp_path / "test.txt")
    write_dataset(test, *te)
    log, ol, U, I, o = wals_vs_oracle(tmp_path, u, i, v, 16, 2, 64,
                                      extra=("--test_dataset=" + test,
                                             "--test_avg_metrics=auc,p@5,r@10,ap,mse"))
    rec = dict(re.findall(r"recorded metric (\w+@?\d*) = ([-\d.e+]+)", log))
    assert set(rec) == {"test_avg_auc", "test_avg_p@5", "test_avg_r@10", "test_avg_ap",
                        "test_avg_mse"}
    # every metric recomputed by the oracle (dense scores, Metrics.cpp restatement) from the
    # saved factors over every test user (numTestUsers = 0); the saved files carry 9
    # decimals, hence the tolerance
    uid, iid = o.ids(0), o.ids(1)
    L = {}
    for a, b, w in zip(*te):
        if a in set(uid) and b in set(iid):
            L.setdefault(int(np.searchsorted(uid, a)), {})[int(np.searchsorted(iid, b))] = w
    users = sorted(L)
    S = po.test_scores(U, I, users)
    vals = {"auc": [], "p@5": [], "r@10": [], "ap": [], "mse": []}
    for t, uu in enumerate(users):
        lab = np.zeros(len(iid))
        for it, w in L[uu].items():
            lab[it] = w
        vals["auc"].append(po.metric_auc(lab, S[t]))
        vals["p@5"].append(po.metric_precision(lab, S[t], 5))
        vals["r@10"].append(po.metric_recall(lab, S[t], 10))
        vals["ap"].append(po.metric_ap(lab, S[t]))
        vals["mse"].append(po.metric_mse(lab, S[t]))
    for name, v in vals.items():
        assert abs(float(rec["test_avg_" + name]) - np.mean(v)) < 1e-4 * max(1.0, abs(np.mean(v))), name


def clustered(nusers, nitems, nnz, seed, groups=10):
    """Users of group g mostly like items of group g: BPR has something to learn."""
    rng = np.random.default_rng(seed)
    u = rng.integers(0, nusers, nnz)
    same = rng.random(nnz) < 0.8
    i = np.where(same, (rng.integers(0, nitems // groups, nnz) * groups + u % groups) % nitems,
                 rng.integers(0, nitems, nnz))
    return u.astype(np.int64), i.astype(np.int64), np.ones(nnz)


def bpr_pref_rate(tmp_path, dataset, checks, nfactors, trials=10):
    data = str(tmp_path / "bpr.txt")
    write_dataset(data, *zip(*[(a, b, 1.0) for a, b in dataset]))
    ok = total = 0
    for t in range(trials):
        uf, itf = str(tmp_path / ("U%d" % t)), str(tmp_path / ("I%d" % t))
        run("bpr", "--train_dataset=" + data, "--nepochs=40", "--nfactors=%d" % nfactors,
            "--init_learning_rate=0.1", "--decay_rate=1.0", "--init_distribution_bound=0.1",
            "--num_negative_samples=1", "--num_hogwild_threads=2", "--use_biases=false",
            "--eval_num_neg=1", "--seed=%d" % (t + 1), "--user_factors=" + uf,
            "--item_factors=" + itf)
        ui, U = read_factors(uf)
        ii, I = read_factors(itf)
        uix = {int(x): n for n, x in enumerate(ui)}
        iix = {int(x): n for n, x in enumerate(ii)}
        for uu, p, n in checks:
            total += 1
            ok += float(U[uix[uu]] @ (I[iix[p]] - I[iix[n]])) > 0
    return ok / total


def test_bpr_cli_learns_preferences(tmp_path):
    # BPREngineTest.cpp:80-157: > 90% of the preference checks hold
    assert bpr_pref_rate(tmp_path, [(1, 1), (2, 2)], [(1, 1, 2), (2, 2, 1)], 1) > 0.9
    ds = [(1, 1), (1, 3), (2, 2), (3, 1)]
    ck = [(1, 1, 2), (1, 3, 2), (2, 2, 1), (2, 2, 3), (3, 1, 2), (3, 3, 2)]
    assert bpr_pref_rate(tmp_path, ds, ck, 1) > 0.9
    assert bpr_pref_rate(tmp_path, ds, ck, 3) > 0.9


def sgd_simulation(uidx, iidx, nitems, k, epochs, lr, decay, lam, bound, use_biases, ev, tev,
                   seed, num_neg=3):
    """Serial reference SGD (oracle BPREngine::update over every positive × num_neg
    rejection-sampled negatives, shuffled after each epoch, lr decay) → per-epoch mean eval
    losses on the given triplet sets."""
    rng = np.random.default_rng(seed)
    nu = int(uidx.max()) + 1
    U = rng.uniform(-bound, bound, (nu, k))
    I = rng.uniform(-bound, bound, (nitems, k))
    b = rng.uniform(-bound, bound, nitems) if use_biases else np.zeros(nitems)
    pos = set((uidx * nitems + iidx).tolist())
    order = np.arange(len(uidx))
    out = []
    for e in range(epochs):
        uu = np.repeat(uidx[order], num_neg)
        pp = np.repeat(iidx[order], num_neg)
        nn = rng.integers(0, nitems, len(uu))
        bad = np.array([x in pos for x in (uu * nitems + nn).tolist()])
        while bad.any():
            nn[bad] = rng.integers(0, nitems, int(bad.sum()))
            bad[bad] = [x in pos for x in (uu[bad] * nitems + nn[bad]).tolist()]
        po.bpr_update_seq(U, I, b, np.stack([uu, pp, nn], 1), lr, *lam, use_biases)
        out.append((po.bpr_loss_sum(U, I, b, ev, use_biases) / len(ev),
                    po.bpr_loss_sum(U, I, b, tev, use_biases) / len(tev)))
        lr *= decay
        order = rng.permutation(order)
    return out


@pytest.mark.parametrize("precision", [32, 64])
def test_bpr_cli_eval_losses_match_oracle(tmp_path, precision):
    """Exact: the logged evaluation losses equal the oracle's loss over the reference's
    evaluation sets on the saved factors.  Statistical: the per-epoch loss trajectory of
    the device Hogwild epochs tracks a serial reference-SGD simulation."""
    u, i, v = clustered(2000, 500, 30000, seed=8)
    te = clustered(2000, 500, 5000, seed=80)
    data, test = str(tmp_path / "tr.txt"), str(tmp_path / "te.txt")
    write_dataset(data, u, i, v)
    write_dataset(test, *te)
    uf, itf = str(tmp_path / "U"), str(tmp_path / "I")
    hp = dict(epochs=8, lr=0.1, decay=0.9, lam=(1.0, 0.025, 0.0025), bound=0.1)
    log = run("bpr", "--train_dataset=" + data, "--test_dataset=" + test,
              "--nepochs=%d" % hp["epochs"], "--nfactors=16", "--use_biases", "--seed=3",
              "--init_learning_rate=%r" % hp["lr"], "--decay_rate=%r" % hp["decay"],
              "--init_distribution_bound=%r" % hp["bound"], "--precision=%d" % precision,
              "--user_factors=" + uf, "--item_factors=" + itf)
    pairs = [(float(a), float(b)) for a, b in
             re.findall(r"train loss = ([-\d.e+]+), test loss = ([-\d.e+]+)", log)]
    assert len(pairs) == hp["epochs"]
    uids, iids, ev, tev = po.bpr_sets(u, i, v, test=te, eval_num_neg=3, eval_seed=42)
    _, U = read_factors(uf)
    _, b, I = read_factors(itf, biases=True)
    assert abs(pairs[-1][0] - po.bpr_loss_sum(U, I, b, ev, True) / len(ev)) < 2e-6
    assert abs(pairs[-1][1] - po.bpr_loss_sum(U, I, b, tev, True) / len(tev)) < 2e-6
    # learning, and close to the serial reference SGD at every epoch
    ui_map = {x: n for n, x in enumerate(uids.tolist())}
    ii_map = {x: n for n, x in enumerate(iids.tolist())}
    sim = sgd_simulation(np.array([ui_map[x] for x in u.tolist()]),
                         np.array([ii_map[x] for x in i.tolist()]), len(iids), 16,
                         hp["epochs"], hp["lr"], hp["decay"], hp["lam"], hp["bound"], True,
                         ev, tev, seed=precision)
    assert pairs[-1][0] < pairs[0][0] - 0.05
    # Hogwild collisions cost most in epoch 1 (large gradients, 500 items); afterwards the
    # device trajectory tracks the serial one closely
    for e, ((dtr, dte), (str_, ste)) in enumerate(zip(pairs, sim)):
        tol = 0.06 if e == 0 else 0.02
        assert abs(dtr - str_) < tol and abs(dte - ste) < tol, (e, pairs, sim)


def test_bpr_cli_test_metrics_with_biases(tmp_path):
    # bpr's evaluation adds the item biases (Engine.cpp:84-86); every test user sampled
    # (num_test_users=0).  Oracle metrics from the saved factors (9 decimals).
    u, i, _ = clustered(300, 120, 6000, seed=4)
    data, test = str(tmp_path / "bpr.txt"), str(tmp_path / "test.txt")
    write_dataset(data, u, i, np.ones(len(u)))
    tu, ti, _ = clustered(300, 120, 900, seed=40)
    write_dataset(test, tu, ti, np.ones(len(tu)))
    uf, itf = str(tmp_path / "U"), str(tmp_path / "I")
    log = run("bpr", "--train_dataset=" + data, "--test_dataset=" + test, "--nepochs=3",
              "--nfactors=12", "--use_biases=true", "--init_distribution_bound=0.1",
              "--test_avg_metrics=auc,p@5,ap,mse", "--seed=3", "--precision=64",
              "--user_factors=" + uf, "--item_factors=" + itf)
    rec = dict(re.findall(r"recorded metric (\w+@?\d*) = ([-\d.e+]+)", log))
    assert set(rec) == {"test_avg_auc", "test_avg_p@5", "test_avg_ap", "test_avg_mse"}
    ui, U = read_factors(uf)
    ii, b, I = read_factors(itf, biases=True)
    uix = {int(x): n for n, x in enumerate(ui)}   # file order = the engine's idx order
    iix = {int(x): n for n, x in enumerate(ii)}
    L = {}
    for a, c in zip(tu, ti):
        if int(a) in uix and int(c) in iix:
            L.setdefault(uix[int(a)], {})[iix[int(c)]] = 1.0
    users = sorted(L)
    S = po.test_scores(U, I, users, b)
    vals = {"auc": [], "p@5": [], "ap": [], "mse": []}
    for t, uu in enumerate(users):
        lab = np.zeros(len(ii))
        lab[list(L[uu])] = 1.0
        vals["auc"].append(po.metric_auc(lab, S[t]))
        vals["p@5"].append(po.metric_precision(lab, S[t], 5))
        vals["ap"].append(po.metric_ap(lab, S[t]))
        vals["mse"].append(po.metric_mse(lab, S[t]))
    for name, v in vals.items():
        assert abs(float(rec["test_avg_" + name]) - np.mean(v)) < 1e-4 * max(1.0, abs(np.mean(v))), name


def test_wals_cli_ngpus_beyond_the_visible_gpus_fails_loudly(tmp_path):
    """--ngpus N splits the rows over N GPUs of this process (qmfx_dist_init_all); asking
    for more GPUs than are visible aborts with the reference's CHECK convention instead of
    quietly running on fewer."""
    import qmf_amd
    n = qmf_amd.device_count() + 1
    u, i, v = load_tiny()
    train = str(tmp_path / "train.txt")
    write_dataset(train, u, i, v)
    r = subprocess.run([os.path.join(BIN, "wals"), "--train_dataset=" + train, "--nepochs=1",
                        "--nfactors=8", "--ngpus=%d" % n, "--user_factors=" + str(tmp_path / "u"),
                        "--item_factors=" + str(tmp_path / "i")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "--ngpus %d" % n in r.stderr and "visible" in r.stderr, r.stderr[-2000:]


def test_wals_cli_ngpus_one_is_the_plain_path(tmp_path):
    """--ngpus 1 (the default) is the single-context path: identical files."""
    u, i, v = load_tiny()
    train = str(tmp_path / "train.txt")
    write_dataset(train, u, i, v)
    dist = str(tmp_path / "init.txt")
    write_dist(dist, np.random.default_rng(3).uniform(-0.01, 0.01, 1000 * 8))
    outs = []
    for flag in ([], ["--ngpus=1"]):
        tag = "n%d" % len(flag)
        run("wals", "--train_dataset=" + train, "--nepochs=2", "--nfactors=8",
            "--distribution_file=" + dist, "--user_factors=" + str(tmp_path / (tag + "u")),
            "--item_factors=" + str(tmp_path / (tag + "i")), *flag)
        outs.append(open(tmp_path / (tag + "u")).read() + open(tmp_path / (tag + "i")).read())
    assert outs[0] == outs[1]
