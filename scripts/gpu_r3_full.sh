#!/bin/bash
# One gpurun call at a code commit: the whole GPU suite, smoke, bench (+ its PMC passes), the rocprof
# kernel trace of the bench, SQ/TCC counters of the metric kernels, UPDATE shapes, BASELINE layers.
# Every GPU step has its own time limit; a fault / abort / timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "FATAL rc=$1 in $2"; exit "$1"; fi; }
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/pytest_gpu.log; fatal $rc pytest
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; fatal $rc smoke
timeout -k 10 600 python bench.py --pmc-dir gpurun_out/pmc > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/bench.log | tail -1 > gpurun_out/bench.json; fatal $rc bench
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run \
  -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pmc > gpurun_out/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; fatal $rc prof
timeout -k 10 420 python scripts/pmc_sq.py gpurun_out/pmc_sq > gpurun_out/pmc_sq.log 2>&1
rc=$?; echo "pmcsq rc=$rc"; tail -2 gpurun_out/pmc_sq.log | cut -c1-600; fatal $rc pmcsq
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mmprof -o run -- python3 scripts/mm_probe.py --shapes cora --sweep mm_split=1,2,4,6,8,11,16,22 > gpurun_out/mm_cora.log 2>&1
rc=$?; echo "mm cora rc=$rc"; fatal $rc mm_cora
timeout -k 10 300 python scripts/mm_probe.py --shapes mid,big --sweep mm_ring_depth=0,3,4,8 > gpurun_out/mm_mid.log 2>&1
rc=$?; echo "mm mid rc=$rc"; fatal $rc mm_mid
timeout -k 10 300 python scripts/mm_probe.py --shapes gin --sweep mm_ring_fr=1,2 > gpurun_out/mm_gin.log 2>&1
rc=$?; echo "mm gin rc=$rc"; fatal $rc mm_gin
timeout -k 10 300 python scripts/mm_probe.py --shapes gin mm_ring=0 > gpurun_out/mm_gin_rows.log 2>&1
rc=$?; echo "mm gin rows rc=$rc"; fatal $rc mm_gin_rows
timeout -k 10 600 python scripts/layer_bench.py > gpurun_out/layers.log 2>&1
rc=$?; echo "layers rc=$rc"; tail -12 gpurun_out/layers.log; fatal $rc layers
echo "gpu_r3_full done"
