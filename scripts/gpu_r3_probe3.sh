#!/bin/bash
# GEMM epilogue with the SF switch hoisted (code size): update_mm tests, then the short-K / Cora /
# GIN / Reddit shapes; Cora split variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { if [ "$1" -ne 0 ]; then echo "FATAL rc=$1 in $2"; exit "$1"; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -k "update_mm" -x > gpurun_out/pytest_mm.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_mm.log; fatal $rc pytest
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/e0 -o run -- python3 scripts/mm_probe.py --shapes short_k,cora_x mm_split=0 > gpurun_out/e0.log 2>&1
rc=$?; echo "e0 rc=$rc"; grep '^{' gpurun_out/e0.log | cut -c1-200; fatal $rc e0
timeout -k 10 200 python3 scripts/mm_probe.py --shapes cora_x --sweep mm_split=4,6,8,10,14,22 > gpurun_out/e1.log 2>&1
rc=$?; echo "e1 rc=$rc"; grep '^{' gpurun_out/e1.log | cut -c1-200; fatal $rc e1
timeout -k 10 200 python3 scripts/mm_probe.py --shapes cora_x --sweep mm_split=4,6,8,10,14,22 mm_ring_fr=1 mm_ring_depth=4 > gpurun_out/e2.log 2>&1
rc=$?; echo "e2 rc=$rc"; grep '^{' gpurun_out/e2.log | cut -c1-200; fatal $rc e2
timeout -k 10 200 python3 scripts/mm_probe.py --shapes cora,gin,big,mid > gpurun_out/e3.log 2>&1
rc=$?; echo "e3 rc=$rc"; grep '^{' gpurun_out/e3.log | cut -c1-200; fatal $rc e3
echo done
