mkdir -p gpurun_out/r02
timeout -k 10 300 python -u bench.py --config c2 --steps 5 --warmup 1 > gpurun_out/r02/c2_v3.json 2> gpurun_out/r02/c2_v3.err
timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 > gpurun_out/r02/c3_f32_v3.json 2> gpurun_out/r02/c3_f32_v3.err
timeout -k 10 300 python -u bench.py --config c2 --precision 64 --steps 5 --warmup 1 --cpu-baseline none > gpurun_out/r02/c2_f64_v3.json 2> gpurun_out/r02/c2_f64_v3.err
for f in c2_v3 c3_f32_v3 c2_f64_v3; do python3 -c "
import json; d=json.load(open('gpurun_out/r02/$f.json')); print('$f', d['ms_per_step'], d['value'], d['roofline']['kernel'], d['roofline']['frac'], d['parity']['max_rel_err'], d.get('cpu_baseline',{}).get('value'))"; done
