cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r6a.log 2>&1; rc=$?; echo "gpu suite rc=$rc"; tail -3 gpurun_out/pytest_gpu_r6a.log; fatal $rc && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r6a.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke_r6a.log; fatal $rc && exit $rc
PMC_GROUPS=tex,l2 timeout -k 10 400 python scripts/pmc_sq.py gpurun_out/pmc_pf0 > gpurun_out/pmc_pf0.log 2>&1; rc=$?; echo "pmc pf0 rc=$rc"; fatal $rc && exit $rc
PMC_GROUPS=tex,l2 timeout -k 10 400 python scripts/pmc_sq.py gpurun_out/pmc_pf1 --knobs seg_pf=1 > gpurun_out/pmc_pf1.log 2>&1; rc=$?; echo "pmc pf1 rc=$rc"
true
