"""End-to-end timing of the drop-in `wals` CLI on a BASELINE-sized text file (VERDICT r05
next #4): the phases that are not epochs — text parse, device grouping, saveFactors — next to
the epochs, and the reference-structure port's reader and grouping on the same file.

  python tools/bench_cli.py [--config c2] [--nepochs 1] [--precision 32] [--out FILE]

Steps (all on the GPU box, files under $TMPDIR):
  1. `qmf_tool gen-dataset`: C2's matrix as `u i w` text (1M users × 100K items, 50M distinct
     pairs, w in 1..5, seed 2) and `gen_uniform`'s distribution file for the item factors;
  2. `qmf_amd/bin/wals` with the reference's flags and QMF_TIMINGS=1: its "timing:" lines give
     parse (DatasetReader::readAll, whole-file parallel parser), init (WALSEngine::init: device
     grouping qmfx_group_signals + CSR + factor upload), optimize (the epochs) and save (both
     factor files, %.9f), and the process wall time is measured around it;
  3. the port's side (reference structure, one thread as the reference's reader is): the
     getline + sscanf loop (`qmf_tool read-seq`, qmf/DatasetReader.cpp:29-59) and the
     oracle's grouping (sort + IdIndex, WALSEngine.cpp:130-163 restated) on the same pairs.
Prints one JSON line (and writes it to --out)."""
import argparse
import json
import os
import re
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "qmf_amd", "bin")
CONFIGS = {"c2": (1_000_000, 100_000, 50_000_000, 64, 2),
           "c3": (10_000_000, 1_000_000, 500_000_000, 128, 3),
           "small": (200_000, 50_000, 10_000_000, 64, 5)}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def run(cmd, env=None, timeout=900):
    t0 = time.perf_counter()
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)
    dt = time.perf_counter() - t0
    if r.returncode != 0:
        log(r.stdout[-2000:], r.stderr[-2000:])
        raise SystemExit("%s failed (%d)" % (cmd[0], r.returncode))
    return r, dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--nepochs", type=int, default=1)
    ap.add_argument("--precision", type=int, default=32, choices=(32, 64))
    ap.add_argument("--no-port", action="store_true")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    nu, ni, nnz, k, seed = CONFIGS[args.config]
    tmp = tempfile.mkdtemp(prefix="qmf_cli_")
    data, dist = os.path.join(tmp, "train.txt"), os.path.join(tmp, "uniform.dat")
    uf, itf = os.path.join(tmp, "user.txt"), os.path.join(tmp, "item.txt")
    try:
        _, t_gen = run([os.path.join(BIN, "qmf_tool"), "gen-dataset", str(nu), str(ni), str(nnz),
                        str(seed), data])
        run([os.path.join(BIN, "gen_uniform"), str(ni * k), str(seed + 100), dist])
        size = os.path.getsize(data)
        log("dataset: %d lines, %.2f GB in %.1f s" % (nnz, size / 1e9, t_gen))
        env = dict(os.environ, QMF_TIMINGS="1")
        cmd = [os.path.join(BIN, "wals"), "--train_dataset=" + data, "--nfactors=%d" % k,
               "--nepochs=%d" % args.nepochs, "--regularization_lambda=0.05",
               "--confidence_weight=40", "--distribution_file=" + dist,
               "--user_factors=" + uf, "--item_factors=" + itf, "--nthreads=16",
               "--precision=%d" % args.precision]
        r, wall = run(cmd, env=env)
        err = r.stderr
        ph = {}
        for name in ("parse", "init", "optimize", "save"):
            m = re.search(r"timing: %s ([0-9.eE+-]+) s" % name, err)
            ph[name] = float(m.group(1)) if m else None
        saved = int(re.search(r"timing: save [0-9.eE+-]+ s, (\d+) bytes", err).group(1))
        losses = [float(x) for x in re.findall(r"train loss = ([0-9.eE+-]+)", err)]
        out = {
            "what": "drop-in wals CLI end to end (%s: %d x %d, %d lines, k=%d, fp%d, %d epoch%s)"
                    % (args.config, nu, ni, nnz, k, args.precision, args.nepochs,
                       "" if args.nepochs == 1 else "s"),
            "command": " ".join(os.path.basename(c) if i == 0 else c for i, c in enumerate(cmd)),
            "file_bytes": size, "wall_s": round(wall, 3),
            "phases_s": {kk: (round(v, 3) if v is not None else None) for kk, v in ph.items()},
            "parse_gb_per_s": round(size / ph["parse"] / 1e9, 3),
            "parse_lines_per_s": round(nnz / ph["parse"], 1),
            "ms_per_epoch": round(ph["optimize"] / args.nepochs * 1e3, 2),
            "save_mb_per_s": round(saved / ph["save"] / 1e6, 1), "saved_bytes": saved,
            "losses": losses,
            "other_s": round(wall - sum(v for v in ph.values() if v), 3),
            "host_threads": 16,
        }
        if not args.no_port:
            # the reference's reader (one thread) on the same file, then its grouping
            # (the oracle's sort + IdIndex restatement) on the parsed pairs
            r2, _ = run([os.path.join(BIN, "qmf_tool"), "read-seq", data])
            lines, t_read = r2.stdout.split()
            import numpy as np
            import pandas as pd
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import pyoracle as po
            df = pd.read_csv(data, sep=" ", header=None, names=["u", "i", "w"], engine="c",
                             dtype={"u": np.int64, "i": np.int64, "w": np.float64})
            t0 = time.perf_counter()
            o = po.OracleWALS(df["u"].to_numpy(), df["i"].to_numpy(), df["w"].to_numpy(), k,
                              0.05, 40.0)
            t_group = time.perf_counter() - t0
            del o, df
            out["port"] = {"readAll_s": float(t_read), "lines": int(lines),
                           "readAll_gb_per_s": round(size / float(t_read) / 1e9, 3),
                           "group_s": round(t_group, 3),
                           "note": "reference-structure port, one thread: getline + sscanf per "
                                   "line (qmf_tool read-seq) and the oracle's sort + IdIndex "
                                   "grouping"}
            out["speedup_parse_plus_init"] = round((float(t_read) + t_group) /
                                                   (ph["parse"] + ph["init"]), 1)
    finally:
        for f in (data, dist, uf, itf):
            if os.path.exists(f):
                os.remove(f)
        os.rmdir(tmp)
    line = json.dumps(out)
    print(line, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
