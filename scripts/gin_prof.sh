#!/bin/bash
# Kernel trace of the GIN products layer (scripts/layer_bench.py), once as built and once with
# GIN's sum handed to the fused MLP in fp32 (--no-bf16-sum): the ABI 10 A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gin_bf -o run -- python3 scripts/layer_bench.py gin-products > gpurun_out/prof_gin_bf.log 2>&1 || exit $?
if [ -z "$GIN_PROF_ONE" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gin_f32 -o run -- python3 scripts/layer_bench.py gin-products --no-bf16-sum > gpurun_out/prof_gin_f32.log 2>&1 || exit $?
fi
grep -h "^gin-products" gpurun_out/prof_gin_*.log | cut -c1-300
