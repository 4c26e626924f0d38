cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "scalar_prefetch or kernel_forms" -x -q --timeout 240 --timeout-method thread > gpurun_out/t_pf2.log 2>&1; rc=$?; echo "pf tests rc=$rc"; tail -2 gpurun_out/t_pf2.log; fatal $rc && exit $rc
if [ $rc -eq 0 ]; then
timeout -k 10 400 python -u scripts/metric_ab.py --rounds 5 20 20:seg_pf=1 20:seg_pf=2 20:seg_pf=3 20:seg_pf=4 > gpurun_out/metric_ab_pf2.log 2>&1; rc=$?; echo "ab rc=$rc"; grep '^{' gpurun_out/metric_ab_pf2.log | cut -c1-120; fatal $rc && exit $rc
fi
HSA_ENABLE_INTERRUPT=0 GTA_DIST_BACKEND=gloo GTA_SINGLE_DEVICE=1 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 8 --steps 3 --warmup 1 --mode edges > gpurun_out/bench_8rank_rehearsal_nointr.log 2>&1; echo "rehearsal rc=$?"; grep '^{' gpurun_out/bench_8rank_rehearsal_nointr.log | cut -c1-300
true
