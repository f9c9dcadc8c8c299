set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s3
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/s3/gputest.log 2>&1 && echo tests ok &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s3/smoke.log 2>&1 && echo smoke ok &&
timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 > gpurun_out/s3/c3_f32.json 2> gpurun_out/s3/c3_f32.err && cat gpurun_out/s3/c3_f32.json
