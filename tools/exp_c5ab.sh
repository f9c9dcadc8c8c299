set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for mode in nowhiten whiten; do
  if [ $mode = nowhiten ]; then export QMFX_NO_WHITEN=1; else unset QMFX_NO_WHITEN; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/p5$mode -o run -- python3 bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/c5$mode.json 2> gpurun_out/c5$mode.err || exit 1
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/p5$mode/run_kernel_trace.csv')):
  n=r['Kernel_Name']
  if 'wals_big' in n or 'woodbury' in n: print('$mode', n[:40], (int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e6, int(r['Grid_Size_X'])//int(r['Workgroup_Size_X']))
"
done
