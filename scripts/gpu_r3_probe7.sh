#!/bin/bash
# k_mm_ring fragment prefetch (mm_ring_pf): bitwise tests, then A/B at depth 3 (3 blocks/CU) and 4 (2/CU).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { if [ "$1" -ne 0 ]; then echo "FATAL rc=$1 in $2"; exit "$1"; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -k "update_mm_ring_bitwise" -x > gpurun_out/pytest_p7.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_p7.log; fatal $rc pytest
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/p7a -o run -- python3 scripts/mm_probe.py --shapes big,mid --sweep mm_ring_pf=0,1 > gpurun_out/p7a.log 2>&1
rc=$?; echo "p7a rc=$rc"; grep '^{' gpurun_out/p7a.log | cut -c1-150; fatal $rc p7a
timeout -k 10 300 python3 scripts/mm_probe.py --shapes big --sweep mm_ring_pf=0,1 mm_ring_depth=4 > gpurun_out/p7b.log 2>&1
rc=$?; echo "p7b rc=$rc"; grep '^{' gpurun_out/p7b.log | cut -c1-150; fatal $rc p7b
echo done
