"""Device test-set evaluation throughput (qmfx_eval_ranks) at a C3-like shape: 1000 test
users × 1M items, k=128, fp32 factors, 10 labelled positives per user.  Prints one JSON line:
scores/s (test users × items per second) and the fp64 VALU roofline of eval_rank_kernel
(one rounded multiply + one rounded add per factor, so the peak for this instruction mix is
half the 78.6 TFLOP/s FMA peak)."""
import json
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import qmf_amd  # noqa: E402


def main():
    nu, ni, k, nt = 100_000, 1_000_000, 128, 1000
    npos = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    rng = np.random.default_rng(0)
    users = rng.choice(nu, nt, replace=False)
    items = np.concatenate([np.sort(rng.choice(ni, npos, replace=False)) for _ in range(nt)])
    rowptr = np.arange(nt + 1, dtype=np.int64) * npos
    with qmf_amd.Context(k, 32) as c:
        c.set_shape(nu, ni)
        c.fill_uniform(0, 0.5, 1)
        c.fill_uniform(1, 0.5, 2)
        c.eval_set_labels(users, rowptr, items, np.ones(len(items)))
        c.eval_ranks()
        reps = 5
        t0 = time.perf_counter()
        for _ in range(reps):
            c.eval_ranks()
        dt = (time.perf_counter() - t0) / reps
    flops = 2.0 * nt * ni * k
    out = {"metric": "test-set ranking statistics (mse/auc/ap/p@k/r@k inputs)",
           "value": nt * ni / dt, "unit": "scores/s", "ms_per_eval": dt * 1e3,
           "config": {"ntest": nt, "nitems": ni, "nfactors": k, "positives_per_user": npos,
                      "precision": "f32 storage, f64 scores"},
           "roofline": {"bound": "fp64 valu", "achieved": flops / dt / 1e12,
                        "peak": 39.3, "unit": "TFLOP/s (mul+add, unfused)",
                        "frac": flops / dt / 1e12 / 39.3}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
