#!/bin/bash
# Cached sibling-weight concatenation (executor._sibling_cat): executor/config tests, then the layers
# that read one (GAT, GraphSAGE, PNA-trans) timed.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { if [ "$1" -ne 0 ]; then echo "FATAL rc=$1 in $2"; exit "$1"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_executor.py tests/test_gpu_configs.py -q -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider -x > gpurun_out/pytest_p10.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_p10.log; fatal $rc pytest
timeout -k 10 400 python scripts/layer_bench.py gcn-cora gat8-flickr gat8-flickr-trans pna-flickr sage-reddit gat8-reddit > gpurun_out/p10_layers.log 2>&1
rc=$?; echo "layers rc=$rc"; grep -o '^[a-z0-9-]* \|"ms_per_forward": [0-9.]*' gpurun_out/p10_layers.log; fatal $rc layers
timeout -k 10 200 python scripts/layer_bench.py gcn-cora gat8-flickr gat8-flickr-trans > gpurun_out/p10_layers2.log 2>&1
rc=$?; echo "layers2 rc=$rc"; grep -o '^[a-z0-9-]* \|"ms_per_forward": [0-9.]*' gpurun_out/p10_layers2.log; fatal $rc layers2
echo done
