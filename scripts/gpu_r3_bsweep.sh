#!/bin/bash
# Column-block count of the metric aggregate re-swept on the round-3 kernels (interleaved, two passes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
for pass in 1 2; do
for B in 18 20 22 24; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 --blocks $B --no-pmc --no-cpu-baseline > gpurun_out/bs_${B}_$pass.log 2>&1
  rc=$?; echo "B=$B pass $pass rc=$rc $(grep '^{' gpurun_out/bs_${B}_$pass.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],4), round(d["value"]/1e9,3))')"
  [ $rc -eq 0 ] || exit $rc
done; done
