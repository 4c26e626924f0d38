#!/bin/bash
# Column-block sweep of the metric on the round-5 kernels: bench.py --blocks B, two interleaved passes
# (each run its own process; no PMC, no CPU baseline, no layers).
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/metric_b_sweep_r05.log
for pass in 1 2; do
  for B in 16 18 20 22 24; do
    timeout -k 10 120 python -u bench.py --blocks $B --no-pmc --no-cpu-baseline --layers none --steps 50 > gpurun_out/b.json 2> gpurun_out/b.err || exit 1
    python -c "import json; b=json.load(open('gpurun_out/b.json')); print(json.dumps({'pass': $pass, 'B': $B, 'ms_per_step': b['ms_per_step'], 'value': b['value']}))" >> gpurun_out/metric_b_sweep_r05.log
  done
done
cat gpurun_out/metric_b_sweep_r05.log
