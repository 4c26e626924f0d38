#!/bin/bash
# Split-K default (64-row groups, 4-deep ring) checked and timed; every BASELINE layer timed.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { if [ "$1" -ne 0 ]; then echo "FATAL rc=$1 in $2"; exit "$1"; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -k "update_mm" -x > gpurun_out/pytest_mm.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_mm.log; fatal $rc pytest
timeout -k 10 200 python3 scripts/mm_probe.py --shapes cora,cora_x > gpurun_out/f0.log 2>&1
rc=$?; echo "f0 rc=$rc"; grep '^{' gpurun_out/f0.log | cut -c1-200; fatal $rc f0
timeout -k 10 600 python scripts/layer_bench.py > gpurun_out/layers.log 2>&1
rc=$?; echo "layers rc=$rc"; grep -v amdgpu.ids gpurun_out/layers.log | cut -c1-60,400-470; fatal $rc layers
echo done
