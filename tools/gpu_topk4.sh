#!/bin/bash
# top-k parity tests, then the default c4 bench (3 sweeps, top-30 over all users) at G = 8 and G = 4
set -e
TAG=${1:-tk}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "topk or transform" --timeout 200 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
timeout -k 10 400 python -u bench.py --no-cpu > gpurun_out/bench_c4_$TAG.json 2> gpurun_out/bench_c4_$TAG.err
ALBEDO_TOPK_SCAN=shared timeout -k 10 400 python -u bench.py --no-cpu > gpurun_out/bench_c4g4_$TAG.json 2> gpurun_out/bench_c4g4_$TAG.err
echo all-ok
