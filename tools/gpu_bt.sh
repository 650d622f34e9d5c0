#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
rm -f gpurun_out/batchtime.txt
for SV in 16 8 4 2 1; do
  D=$((24576 / (SV * 256)))
  timeout -k 10 120 ./tools/probe/batchtime 256 $SV 20000 8192 $D >> gpurun_out/batchtime.txt 2>&1
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu -k "nnls" > gpurun_out/nnls_q.log 2>&1
echo all-ok
