cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "mm_wave or update_mm_hand or ring_bitwise or mm_vector" -x -v --timeout 240 --timeout-method thread > gpurun_out/t_mmwave.log 2>&1; echo "mm tests rc=$?"; tail -3 gpurun_out/t_mmwave.log
timeout -k 10 300 python -u scripts/mm_wave_ab.py --rounds 3 232965,602,128 29000,602,128 44625,500,128 899756,500,128 89250,500,128 29000,602,256 > gpurun_out/mm_wave_ab.log 2>&1; echo "mm ab rc=$?"
HSA_ENABLE_INTERRUPT=0 timeout -k 10 200 python -u scripts/setup_stall_probe.py --iters 2 --limit 170 > gpurun_out/stall_probe_nointr.log 2>&1; echo "probe nointr rc=$?"
tail -1 gpurun_out/stall_probe_nointr.log | grep -q "stuck at the limit: \[\]" && { timeout -k 10 200 python -u scripts/setup_stall_probe.py --iters 2 --limit 170 > gpurun_out/stall_probe_default.log 2>&1; echo "probe default rc=$?"; }
true
