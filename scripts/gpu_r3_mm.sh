#!/bin/bash
# GEMM experiments: correctness of the ring forms, then split-K variants for GCN Cora's layer-1 shape
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "FATAL rc=$1 in $2"; exit "$1"; fi; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider -k "update_mm or ring or split or bf16" > gpurun_out/pytest_mm.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_mm.log; fatal $rc pytest
i=0
for cfg in "--sweep mm_split=6,8,10,11" "--sweep mm_split=8,11,16,22 mm_ring_depth=3" "--sweep mm_split=8,11,16 mm_ring_depth=4" \
           "--sweep mm_split=4,6,8,11 mm_ring_fr=1" "--sweep mm_split=8,11,16 mm_ring=0"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/mmx$i -o run -- python3 scripts/mm_probe.py --shapes cora_x $cfg > gpurun_out/mmx$i.log 2>&1
  rc=$?; echo "mmx$i [$cfg] rc=$rc"; grep '^{' gpurun_out/mmx$i.log | cut -c1-160; fatal $rc mmx$i
done
timeout -k 10 200 python scripts/mm_probe.py --shapes gin,big > gpurun_out/mm_gin2.log 2>&1
rc=$?; echo "gin2 rc=$rc"; grep '^{' gpurun_out/mm_gin2.log | cut -c1-170
