#!/bin/bash
# k_mm_ring grid: persistent (every CU slot, groups strided over blocks) vs one block per row group
# (the dispatcher balances groups over CUs), at the default depth and at 4 stages.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { if [ "$1" -ne 0 ]; then echo "FATAL rc=$1 in $2"; exit "$1"; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -k "update_mm_ring_bitwise or default_is_the_ring" -x > gpurun_out/pytest_p6.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_p6.log; fatal $rc pytest
timeout -k 10 300 python3 scripts/mm_probe.py --shapes big,mid --sweep mm_ring_persist=1,0 > gpurun_out/p6a.log 2>&1
rc=$?; echo "p6a rc=$rc"; grep '^{' gpurun_out/p6a.log | cut -c1-170; fatal $rc p6a
timeout -k 10 300 python3 scripts/mm_probe.py --shapes big --sweep mm_ring_persist=1,0 mm_ring_depth=4 > gpurun_out/p6b.log 2>&1
rc=$?; echo "p6b rc=$rc"; grep '^{' gpurun_out/p6b.log | cut -c1-170; fatal $rc p6b
echo done
