"""CPU tests of the drop-in C++ host library (qmf_amd/host): its own unit tests (the
reference's qmf/test/*.cpp re-expressed) and its bookkeeping against the oracle's
restatement of the reference, bit-exact: WALS ids + both CSR orientations
(WALSEngine.cpp:130-163) and the BPR indexes + evaluation triplets (BPREngine.cpp:63-131).
No GPU is used."""
import os
import subprocess

import numpy as np
import pytest

import pyoracle as po
from helpers import ROOT, load_ml100k, load_tiny, synth

BIN = os.path.join(ROOT, "qmf_amd", "bin")


@pytest.fixture(scope="module", autouse=True)
def built():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "qmf_amd"), "-j8"], check=True)
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)


def tool(*args):
    out = subprocess.run([os.path.join(BIN, "qmf_tool")] + [str(a) for a in args], check=True,
                         capture_output=True, text=True).stdout
    res = {}
    for line in out.splitlines():
        name, n, *vals = line.split(" ")
        assert int(n) == len(vals)
        res[name] = np.array([float(v) for v in vals]) if name.endswith("val") else \
            np.array([int(v) for v in vals], dtype=np.int64)
    return res


def write_dataset(path, users, items, values):
    with open(path, "w") as f:
        for u, i, v in zip(users, items, values):
            f.write("%d %d %s\n" % (u, i, repr(float(v)) if v != int(v) else int(v)))


def test_host_unit_tests():
    r = subprocess.run([os.path.join(BIN, "qmf_host_tests")], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 failed checks" in r.stdout


def _check_csr_against_oracle(path, users, items, values):
    d = tool("wals-csr", path)
    o = po.OracleWALS(users, items, values, 4)
    assert np.array_equal(d["uids"], o.ids(0)) and np.array_equal(d["iids"], o.ids(1))
    for side, p in ((0, "u"), (1, "i")):
        rp, col, val = o.csr(side)
        assert np.array_equal(d[p + "rowptr"], rp)
        assert np.array_equal(d[p + "col"], col)
        # duplicate (u, i) pairs: the reference's std::sort leaves their order unspecified
        row = np.repeat(np.arange(len(rp) - 1), np.diff(rp))
        a = np.lexsort((val, col, row))
        b = np.lexsort((d[p + "val"], d[p + "col"], row))
        assert np.array_equal(val[a], d[p + "val"][b])


def test_wals_grouping_tiny_fixture(golden_dir):
    u, i, v = load_tiny()
    _check_csr_against_oracle(os.path.join(golden_dir, "tiny.txt"), u, i, v)


def test_wals_grouping_ml100k_shape(tmp_path):
    d = load_ml100k()
    p = str(tmp_path / "ml.txt")
    write_dataset(p, d["users"], d["items"], d["values"])
    _check_csr_against_oracle(p, d["users"], d["items"], d["values"])


def test_wals_grouping_signed_sparse_ids(tmp_path):
    rng = np.random.default_rng(4)
    u, i, v = synth(3000, 800, 20000, seed=4)
    # scatter ids over the signed int64 range, with duplicates and fractional values
    u = (u * 7919 - 10 ** 6) * 1_000_003
    i = i * -(2 ** 40) + 17
    dup = rng.integers(0, len(u), 500)
    u, i = np.concatenate([u, u[dup]]), np.concatenate([i, i[dup]])
    v = np.concatenate([v, rng.integers(0, 6, 500)]) + 0.25
    p = str(tmp_path / "s.txt")
    write_dataset(p, u, i, v)
    _check_csr_against_oracle(p, u, i, v)


@pytest.mark.parametrize("neg,seed", [(3, 42), (1, 7), (5, 123)])
def test_bpr_eval_sets_match_reference_sampling(tmp_path, neg, seed):
    d = load_ml100k()
    n = len(d["users"])
    cut = n * 4 // 5
    tr = (d["users"][:cut], d["items"][:cut], d["values"][:cut])
    te = (d["users"][cut:], d["items"][cut:], d["values"][cut:])
    ptr, pte = str(tmp_path / "tr.txt"), str(tmp_path / "te.txt")
    write_dataset(ptr, *tr)
    write_dataset(pte, *te)
    got = tool("bpr-sets", ptr, pte, neg, seed)
    uids, iids, ev, tev = po.bpr_sets(*tr, test=te, eval_num_neg=neg, eval_seed=seed)
    assert np.array_equal(got["uids"], uids) and np.array_equal(got["iids"], iids)
    assert np.array_equal(got["eval"].reshape(-1, 3), ev)
    assert np.array_equal(got["testeval"].reshape(-1, 3), tev)
    assert len(ev) == neg * int((tr[2] >= 1).sum())


def test_bpr_eval_sets_tiny_values_below_one_dropped(golden_dir):
    u, i, v = load_tiny()
    got = tool("bpr-sets", os.path.join(golden_dir, "tiny.txt"), "-", 2, 42)
    uids, iids, ev, _ = po.bpr_sets(u, i, v, eval_num_neg=2, eval_seed=42)
    assert np.array_equal(got["uids"], uids) and np.array_equal(got["iids"], iids)
    assert np.array_equal(got["eval"].reshape(-1, 3), ev)
    assert len(got["testeval"]) == 0


def test_cli_flags_and_usage():
    for exe in ("wals", "bpr"):
        r = subprocess.run([os.path.join(BIN, exe), "--help"], capture_output=True, text=True)
        assert "train_dataset" in r.stderr and "nfactors" in r.stderr
        r = subprocess.run([os.path.join(BIN, exe), "--no_such_flag=1"], capture_output=True,
                           text=True)
        assert r.returncode != 0 and "unknown command line flag" in r.stderr


def test_cli_without_gpu_fails_loudly(golden_dir, tmp_path):
    # the engines never fall back to the CPU: without a device, init aborts
    r = subprocess.run([os.path.join(BIN, "wals"), "--train_dataset=" +
                        os.path.join(golden_dir, "tiny.txt"), "--nepochs=1", "--nfactors=4"],
                       capture_output=True, text=True, env=dict(os.environ, HIP_VISIBLE_DEVICES="-1")
                       if not os.path.exists("/dev/kfd") else os.environ)
    if os.path.exists("/dev/kfd"):
        pytest.skip("a GPU is present")
    assert r.returncode != 0 and "qmfx_create" in r.stderr


def test_gen_uniform(tmp_path):
    out = str(tmp_path / "u.dat")
    subprocess.run([os.path.join(BIN, "gen_uniform"), "1000", "5", out], check=True)
    x = np.loadtxt(out)
    assert x.shape == (1000,) and np.all(np.abs(x) <= 0.01)
    lines = open(out).read().splitlines()
    assert all(len(s.split(".")[1]) == 9 for s in lines)


def test_cli_ngpus_without_gpus_fails_loudly(golden_dir):
    # --ngpus 2 counts the visible GPUs first: with none (or one) it aborts, never runs on
    # fewer ranks than asked
    if os.path.exists("/dev/kfd"):
        pytest.skip("a GPU is present (tests/test_cli_gpu.py covers this case there)")
    r = subprocess.run([os.path.join(BIN, "wals"), "--train_dataset=" +
                        os.path.join(golden_dir, "tiny.txt"), "--nepochs=1", "--nfactors=4",
                        "--ngpus=2"], capture_output=True, text=True)
    assert r.returncode != 0 and "qmfx_device_count" in r.stderr


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_host_unit_tests_under_sanitizers(kind):
    """the host code (parallel parser, %.9f writer, ParallelExecutor, id
    grouping, metrics, BPR host init) under ASan + UBSan and under TSan.  Any report fails
    the run: ASan/UBSan abort (no recovery), TSan exits 66."""
    exe = os.path.join(BIN, kind, "qmf_host_tests")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1",
               TSAN_OPTIONS="halt_on_error=1:exitcode=66")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert " 0 failed checks" in r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr
