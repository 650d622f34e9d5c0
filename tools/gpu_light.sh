#!/bin/bash
# light/heavy threshold sweep at c4 and c2 (no tests)
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for L in 16 32 48; do
  timeout -k 10 200 python -u bench.py --no-cpu --topk-users 0 --light $L > gpurun_out/bench_c4_L$L.json 2> gpurun_out/bench_c4_L$L.err
done
for L in 0 16; do
  timeout -k 10 100 python -u bench.py --config c2 --steps 5 --no-cpu --topk-users 0 --light $L > gpurun_out/bench_c2_L$L.json 2> gpurun_out/bench_c2_L$L.err
done
echo all-ok
