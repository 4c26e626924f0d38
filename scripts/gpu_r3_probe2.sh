#!/bin/bash
# GEMM probes: the ring GEMMs' DMA lane maps (row-contiguous vs lane = fragment) checked bitwise by the
# update_mm tests, then timed on the GIN / Reddit / Flickr / Cora shapes; Cora split/fragment/depth
# variants with per-kernel times. Every GPU step has its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { if [ "$1" -ne 0 ]; then echo "FATAL rc=$1 in $2"; exit "$1"; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -k "update_mm" > gpurun_out/pytest_mm.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_mm.log; fatal $rc pytest
timeout -k 10 200 python3 scripts/mm_probe.py --shapes gin --sweep mm_dma_rows=0,1 > gpurun_out/gin_dma.log 2>&1
rc=$?; echo "gin rc=$rc"; grep '^{' gpurun_out/gin_dma.log | cut -c1-200; fatal $rc gin
timeout -k 10 200 python3 scripts/mm_probe.py --shapes big --sweep mm_dma_rows=0,1 > gpurun_out/big_dma.log 2>&1
rc=$?; echo "big rc=$rc"; grep '^{' gpurun_out/big_dma.log | cut -c1-200; fatal $rc big
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cora0 -o run -- python3 scripts/mm_probe.py --shapes cora_x --sweep mm_dma_rows=0,1 > gpurun_out/cora0.log 2>&1
rc=$?; echo "cora0 rc=$rc"; grep '^{' gpurun_out/cora0.log | cut -c1-200; fatal $rc cora0
i=0
for cfg in "--sweep mm_split=6,8,10,14 mm_ring_fr=1 mm_ring_depth=4" "--sweep mm_split=6,8,10,14 mm_ring_depth=4" "--sweep mm_split=4,6,8,10 mm_ring_fr=1"; do
  i=$((i+1))
  timeout -k 10 200 python3 scripts/mm_probe.py --shapes cora_x $cfg > gpurun_out/corax$i.log 2>&1
  rc=$?; echo "corax$i [$cfg] rc=$rc"; grep '^{' gpurun_out/corax$i.log | cut -c1-200; fatal $rc corax$i
done
timeout -k 10 200 python3 scripts/mm_probe.py --shapes mid --sweep mm_dma_rows=0,1 > gpurun_out/mid_dma.log 2>&1
rc=$?; echo "mid rc=$rc"; grep '^{' gpurun_out/mid_dma.log | cut -c1-200; fatal $rc mid
echo done
