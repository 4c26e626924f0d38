#!/bin/bash
# K-tail tests of both ring GEMMs; then counters of the fp32 ring at full chip (Reddit x.W) and on
# half the chip (16,384 x 1,433): effective clock (GRBM_GUI_ACTIVE / 8 / time) and MFMA busy.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { if [ "$1" -ne 0 ]; then echo "FATAL rc=$1 in $2"; exit "$1"; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -k "every_k_tail" -x > gpurun_out/pytest_ktail.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_ktail.log; fatal $rc pytest
timeout -k 10 500 python -u -m pytest tests/test_gpu_distributed.py -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider -x > gpurun_out/pytest_dist.log 2>&1
rc=$?; echo "pytest dist rc=$rc"; tail -3 gpurun_out/pytest_dist.log; fatal $rc pytest_dist
for sh in big_one mid_one; do
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/clk_$sh -o run -- python3 scripts/mm_probe.py --shapes $sh > gpurun_out/clk_$sh.log 2>&1
rc=$?; echo "clk $sh rc=$rc"; grep '^{' gpurun_out/clk_$sh.log | cut -c1-200; fatal $rc clk
done
echo done
