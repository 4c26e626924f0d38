#!/bin/bash
# GIN ops 3-4 in one launch (gta_aggregate_self, ABI 7): bitwise checks, tests, then the GIN layer timed.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { if [ "$1" -ne 0 ]; then echo "FATAL rc=$1 in $2"; exit "$1"; fi; }
timeout -k 10 120 python scripts/aggregate_self_probe.py > gpurun_out/dbg2.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/dbg2.log | tail -5; fatal $rc dbg2
timeout -k 10 500 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_executor.py tests/test_gpu_configs.py -q -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider -k "self_term or gin or GIN or executor or config or aggregate" -x > gpurun_out/pytest_p9b.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_p9b.log; fatal $rc pytest
timeout -k 10 300 python scripts/layer_bench.py gin-products > gpurun_out/p9b_layers.log 2>&1
rc=$?; echo "layers rc=$rc"; grep -o '^[a-z0-9-]* \|"ms_per_forward": [0-9.]*' gpurun_out/p9b_layers.log; fatal $rc layers
echo done
