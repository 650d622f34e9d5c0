#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for SV in 16 8 4 2 1; do
  D=$((24576 / (SV * 256)))
  timeout -k 10 120 ./tools/probe/batchtime 256 $SV 20000 8192 $D >> gpurun_out/batchtime.txt 2>&1
done
for M in 16 8 4; do
ALBEDO_NNLS_MINSLOTS=$M timeout -k 10 300 python -u bench.py --config c5 --steps 1 --no-cpu --topk-users 0 > gpurun_out/bench_c5_ms$M.json 2> gpurun_out/bench_c5_ms$M.err
done
echo all-ok
