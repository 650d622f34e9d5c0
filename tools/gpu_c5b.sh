#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --config c5 --steps 2 --no-cpu --topk-users 0 > gpurun_out/bench_c5_$1.json 2> gpurun_out/bench_c5_$1.err
echo all-ok
