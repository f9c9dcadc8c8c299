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
