#!/bin/bash
# Fused output SF of the attention aggregate (ABI 6): its GPU test, the executor stream tests, then
# the GAT layers timed.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { if [ "$1" -ne 0 ]; then echo "FATAL rc=$1 in $2"; exit "$1"; fi; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_executor.py -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -k "fused_output_sf or gat or executor or stream" -x > gpurun_out/pytest_p8.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_p8.log; fatal $rc pytest
timeout -k 10 300 python scripts/layer_bench.py gat8-flickr gat8-reddit gcn-cora > gpurun_out/p8_layers.log 2>&1
rc=$?; echo "layers rc=$rc"; grep -o '^[a-z0-9-]* \|"ms_per_forward": [0-9.]*' gpurun_out/p8_layers.log; fatal $rc layers
echo done
