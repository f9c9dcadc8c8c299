"""bench.py's launcher and rank checks (CPU only: no GPU is touched)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_single_gpu_runs_in_process():
    assert bench.launch_plan(1, {}, ["--steps", "2"]) is None


def test_ranks_run_in_process_under_a_launcher():
    # torch.distributed.run sets WORLD_SIZE: the rank must not launch again
    assert bench.launch_plan(8, {"WORLD_SIZE": "8"}, ["--gpus", "8"]) is None


def test_multi_gpu_relaunches_under_torchrun_as_a_child():
    cmd = bench.launch_plan(4, {}, ["--gpus", "4", "--steps", "3"], port=29511)
    assert cmd[0] == sys.executable
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-port=29511" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == [os.path.abspath(bench.__file__), "--gpus", "4", "--steps", "3"][-4:]


def test_world_mismatch_fails():
    bench.check_world(2, 2)
    with pytest.raises(SystemExit, match="started 1 rank"):
        bench.check_world(2, 1)


def test_more_ranks_than_gpus_fails():
    bench.check_world(2, 2, visible=2, local=1)
    with pytest.raises(SystemExit, match="sees only 1"):
        bench.check_world(2, 2, visible=1, local=1)


def test_gpus_2_without_a_second_gpu_fails_loudly(tmp_path):
    """End to end on a machine with fewer GPUs than --gpus (here: none): the relaunched
    ranks must exit non-zero instead of printing an n_gpus: 1 line."""
    import subprocess
    env = dict(os.environ, QMFX_BENCH_LIMIT_S="60")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--steps", "1", "--warmup", "0", "--cpu-baseline", "none", "--no-parity"],
                       cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert '"n_gpus"' not in r.stdout


def test_cpu_epoch_estimate_is_conservative_at_c3():
    # measured on the GPU box: 355.5 s on 16 threads (profiles/r02)
    est = bench.cpu_epoch_estimate_s(10_000_000, 1_000_000, 500_000_000, 128, 16)
    assert 355.5 < est < 500


def test_work_skipping_env_is_refused():
    """A work-skipping knob in the environment: no line is printed (SystemExit)."""
    with pytest.raises(SystemExit, match="QMFX_ABLATE"):
        bench.check_env({"QMFX_ABLATE": "3"}, "")
    bench.check_env({"QMFX_ABLATE": "0", "QMFX_PIECES": "4"}, "")  # 0 / route knobs are fine


def test_variant_library_is_refused_unless_allowed():
    with pytest.raises(SystemExit, match="timing-variant"):
        bench.check_env({}, "exp1: woodbury.hip -DFOO=1")
    bench.check_env({}, "exp1: woodbury.hip -DFOO=1", allow_variant=True)
    bench.check_env({}, "")


def test_engine_env_reports_qmfx_knobs_only():
    env = {"QMFX_PIECES": "4", "QMFX_BENCH_LIMIT_S": "60", "PATH": "/bin", "QMFX_NO_WHITEN": "1"}
    assert bench.engine_env(env) == {"QMFX_NO_WHITEN": "1", "QMFX_PIECES": "4"}


def test_product_library_is_not_a_variant():
    import qmf_amd
    assert qmf_amd._abi.build_variant() == ""


def _exchange_rank(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # rank r: exchange 10+r ms per half (summed over 2 steps), exposed 1+r, solves 20-r
    stats = {sd: {"exchange_ms": 2 * (10.0 + rank + sd), "exposed_ms": 2 * (1.0 + rank),
                  "solve_ms": 2 * (20.0 - rank), "halves": 2} for sd in (0, 1)}

    def reduce_max(vals):
        t = torch.tensor(vals, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return [float(v) for v in t]
    model = {0: bench.exchange_model(10_000_000, 128, 8, world),
             1: bench.exchange_model(1_000_000, 128, 8, world)}
    q.put((rank, bench.exchange_fields(stats, 2, reduce_max, model)))
    dist.destroy_process_group()


def test_exchange_fields_are_max_over_ranks_gloo_world2():
    """--gpus N lines carry per-half exchange_ms / exposed_ms / solve_ms, the max over ranks
    (the driver's first 8-GPU run must say whether the user half is exchange-bound)."""
    import multiprocessing as mp
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_exchange_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    assert res[0] == res[1]
    f = res[0]
    assert set(f) == {"user_half", "item_half"}
    keys = ("exchange_ms", "exposed_ms", "solve_ms")
    assert {k: f["user_half"][k] for k in keys} == {"exchange_ms": 11.0, "exposed_ms": 2.0,
                                                    "solve_ms": 20.0}
    assert {k: f["item_half"][k] for k in keys} == {"exchange_ms": 12.0, "exposed_ms": 2.0,
                                                    "solve_ms": 20.0}
    # the DESIGN §6 model beside the measurement: C3 fp64 user half, world 2: half of 10.24 GB
    p = f["user_half"]["predicted"]
    assert p["bytes_in_per_rank"] == 10_000_000 * 128 * 8 / 2
    assert abs(p["model_ms_bus"] - 5.12e9 / 350e9 * 1e3) < 1e-3
    assert f["user_half"]["measured_gbs_in_per_rank"] == round(5.12e9 / 11.0 / 1e6, 1)


def _fake_stats(d_ms, w_ms, d_side_ms, w_side_ms):
    """class_stats()-shaped accounting: per class the total and per-side figures (two launches
    per side; the *_side_ms arguments are per launch)."""
    def st(ms, launches, fl, by):
        return dict(ms=ms, launches=launches, flops=fl, bytes=by)
    return {
        "direct": {"total": st(d_ms, 4, 0, 0),
                   "side": {0: st(2 * d_side_ms[0], 2, 2 * 1e9, 2 * 1e9),
                            1: st(2 * d_side_ms[1], 2, 2 * 9.12e12, 2 * 5.3e11)}},
        "whitened": {"total": st(w_ms, 2, 0, 0),
                     "side": {0: st(2 * w_side_ms[0], 2, 2 * 5e11, 2 * 528.3e9),
                              1: st(0, 0, 0, 0)}},
    }


def test_roofline_fields_are_fixed_per_half():
    """both halves are first-class fields; the headline does not flip on a tie
    (C3 fp64: whitened 3531.5 vs direct 3530.4 ms)."""
    st = _fake_stats(3530.4, 3531.5, (0.07, 176.4), (176.6, 0))
    classes = bench.roofline_classes(st, 128, 64, whitened_rows={0: 9_900_000, 1: 0})
    roof = bench.roofline_object(classes)
    assert roof["kernel"] == "wals_direct_kernel" and roof["launch_side"] == 1  # tie → item half
    assert set(roof) >= {"kernel", "bound", "achieved", "peak", "unit", "frac", "launch_ms",
                         "bytes_per_launch", "flops_per_launch", "launch_side", "weakest",
                         "user_half", "item_half"}
    uh, ih = roof["user_half"], roof["item_half"]
    assert uh["kernel"] == "wals_whitened (row solve + unwhiten)" and uh["bound"] == "hbm"
    assert ih["kernel"] == "wals_direct_kernel" and ih["bound"] == "mfma"
    # §8(d) bytes over the launch time, the x' round trip beside them (not inside)
    assert abs(uh["achieved"] - 528.3e9 / 0.1766 / 1e9) < 1.0
    assert uh["extra_bytes"] == 2 * 9_900_000 * 128 * 8
    assert abs(ih["frac"] - 9.12e12 / 0.1764 / 1e12 / bench.PEAK_F64_TFLOPS) < 1e-3
    # a clear winner is named whatever its side
    st2 = _fake_stats(1000.0, 3000.0, (0.07, 500.0), (1500.0, 0))
    roof2 = bench.roofline_object(bench.roofline_classes(st2, 128, 64))
    assert roof2["kernel"] == "wals_whitened (row solve + unwhiten)"
    assert roof2["user_half"]["kernel"] == roof2["kernel"]
