#!/bin/bash
# Round-4 probe 2: XCD placement of a deep grid, L2 hit rates of the line-split forms, then the
# full GPU suite, smoke, bench (N = 1) and the 2-rank bench rehearsal with its per-rank fields.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 60 ./scripts/xcd_probe > gpurun_out/xcd_probe.log 2>&1
rc=$?; echo "xcd_probe rc=$rc"; cat gpurun_out/xcd_probe.log; [ $rc -eq 0 ] || exit $rc
for v in "20 1" "16 2" "8 4"; do
  set -- $v
  PMC_GROUPS=l2 timeout -k 10 200 python scripts/pmc_sq.py gpurun_out/pmc_l2_b$1_x$2 --blocks $1 --knobs seg_xcd=$2 > gpurun_out/pmc_l2_b$1_x$2.log 2>&1
  rc=$?; echo "pmc l2 B=$1 NL=$2 rc=$rc"; tail -1 gpurun_out/pmc_l2_b$1_x$2.log; [ $rc -eq 0 ] || exit $rc
done
STEPS="tests smoke bench bench2" PYTEST_ARGS="--timeout 300 --timeout-method thread" BENCH2_MODES=edges bash scripts/gpu_round.sh
timeout -k 10 300 python -u scripts/gin_ic_probe.py > gpurun_out/gin_ic_probe.log 2>&1
rc=$?; echo "gin_ic_probe rc=$rc"; cat gpurun_out/gin_ic_probe.log | grep '^{'
timeout -k 10 400 python -u scripts/tile_chunks.py --grid 4x2 --rank 0 1 0.5,0.5 0.7,0.3 0.6,0.4 0.55,0.3,0.15 0.5,0.3,0.2 0.6,0.25,0.15 > gpurun_out/tile_chunks.log 2>&1
rc=$?; echo "tile_chunks rc=$rc"; grep '^{' gpurun_out/tile_chunks.log
