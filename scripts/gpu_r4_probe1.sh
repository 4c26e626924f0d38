#!/bin/bash
# Round-4 probe: XCD line-split metric kernel A/B, its bitwise tests, the 32x32 ring GEMM test + A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/metric_ab.py --rounds 3 20 20:seg_xcd=4 20:seg_xcd=2 8:seg_xcd=4 10:seg_xcd=4 12:seg_xcd=4 12:seg_xcd=2 16:seg_xcd=2 > gpurun_out/metric_ab.log 2>&1
rc=$?; echo "metric_ab rc=$rc"; cat gpurun_out/metric_ab.log | grep '^{' ; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_metric.py tests/test_gpu_ops.py -m gpu -x -q --timeout 200 --timeout-method thread -k "xcd or kernel_forms or ring_bitwise or edge_case" > gpurun_out/pytest_probe1.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_probe1.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u scripts/mm_probe.py --shapes big,mid --sweep mm_ring_m32=0,1 > gpurun_out/mm_m32.log 2>&1
rc=$?; echo "mm rc=$rc"; cat gpurun_out/mm_m32.log
