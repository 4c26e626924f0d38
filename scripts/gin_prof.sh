cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gin_bf -o run -- python3 scripts/layer_bench.py gin-products > gpurun_out/prof_gin_bf.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gin_f32 -o run -- python3 scripts/layer_bench.py gin-products --no-bf16-sum > gpurun_out/prof_gin_f32.log 2>&1 || exit $?
grep gin-products gpurun_out/prof_gin_bf.log gpurun_out/prof_gin_f32.log | cut -c1-300
