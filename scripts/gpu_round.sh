#!/bin/bash
# One gpurun call: GPU parity tests -> bench -> rocprofv3 kernel trace.
# Every GPU step has its own time limit; any fault/abort/timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS=${STEPS:-"tests bench prof"}
stop_if_fatal() {  # $1 = rc, $2 = step name; test failures (rc 1) are not fatal
  if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "FATAL rc=$1 in $2; stopping"; exit "$1"; fi
}
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 ${T_TESTS:-700} python -m pytest ${PYTEST_TARGET:-tests} -m gpu -x -q ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
      rc=$?; echo "pytest_gpu rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; stop_if_fatal $rc tests ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
      rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log; stop_if_fatal $rc smoke ;;
    bench)
      timeout -k 10 ${T_BENCH:-600} python bench.py --pmc-dir gpurun_out/pmc ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
      rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log; stop_if_fatal $rc bench ;;
    prof)
      export TMPDIR=/tmp
      timeout -k 10 ${T_PROF:-600} rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run \
        -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pmc --layers none ${BENCH_ARGS} > gpurun_out/prof.log 2>&1
      rc=$?; echo "prof rc=$rc"; tail -3 gpurun_out/prof.log; stop_if_fatal $rc prof ;;
    pmc)
      export TMPDIR=/tmp
      timeout -k 10 ${T_PROF:-600} rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run \
        -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/pmc_fetch.log 2>&1
      rc=$?; echo "pmc fetch rc=$rc"; stop_if_fatal $rc pmc
      timeout -k 10 ${T_PROF:-600} rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run \
        -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/pmc_write.log 2>&1
      rc=$?; echo "pmc write rc=$rc"; stop_if_fatal $rc pmc ;;
    bench2)
      for m in ${BENCH2_MODES:-edges rows}; do
        # several ranks on ONE GPU starve each other for tens of seconds on this pool unless completion
        # signals are polled: rehearsals only; the N-GPU runs keep the default
        HSA_ENABLE_INTERRUPT=0 GTA_DIST_BACKEND=gloo GTA_SINGLE_DEVICE=1 timeout -k 10 ${T_BENCH:-600} python -m torch.distributed.run \
          --nnodes=1 --nproc-per-node ${BENCH2_RANKS:-2} --master-addr 127.0.0.1 --master-port 29511 bench.py \
          --gpus ${BENCH2_RANKS:-2} --steps 3 --warmup 1 --mode $m ${BENCH2_ARGS} > gpurun_out/bench2_$m.log 2>&1
        rc=$?; echo "bench2 $m rc=$rc"; grep '^{' gpurun_out/bench2_$m.log | tail -1; stop_if_fatal $rc bench2
      done ;;
    layers)
      timeout -k 10 ${T_LAYERS:-600} python scripts/layer_bench.py ${LAYER_ARGS} > gpurun_out/layers.log 2>&1
      rc=$?; echo "layers rc=$rc"; tail -6 gpurun_out/layers.log; stop_if_fatal $rc layers ;;
    mm)
      timeout -k 10 ${T_MM:-300} python scripts/mm_probe.py ${MM_ARGS} > gpurun_out/mm_probe.log 2>&1
      rc=$?; echo "mm rc=$rc"; tail -20 gpurun_out/mm_probe.log; stop_if_fatal $rc mm ;;
    pmcsq)
      timeout -k 10 ${T_PMCSQ:-420} python scripts/pmc_sq.py gpurun_out/pmc_sq > gpurun_out/pmc_sq.log 2>&1
      rc=$?; echo "pmcsq rc=$rc"; tail -3 gpurun_out/pmc_sq.log; stop_if_fatal $rc pmcsq ;;
    metricab)
      timeout -k 10 ${T_AB:-400} python -u scripts/metric_ab.py ${AB_ARGS:-20 16} > gpurun_out/metric_ab.log 2>&1
      rc=$?; echo "metricab rc=$rc"; grep '^{' gpurun_out/metric_ab.log; stop_if_fatal $rc metricab ;;
    tile)
      timeout -k 10 ${T_TILE:-400} python -u scripts/tile_chunks.py ${TILE_ARGS} > gpurun_out/tile_chunks.log 2>&1
      rc=$?; echo "tile rc=$rc"; grep '^{' gpurun_out/tile_chunks.log; stop_if_fatal $rc tile ;;
    expr)
      timeout -k 10 ${T_EXPR:-300} python -u scripts/expr_probe.py ${EXPR_ARGS:-128} > gpurun_out/expr_probe.log 2>&1
      rc=$?; echo "expr rc=$rc"; grep '^{' gpurun_out/expr_probe.log; stop_if_fatal $rc expr ;;
    *) echo "unknown step $s";;
  esac
done
echo "gpu_round done"
