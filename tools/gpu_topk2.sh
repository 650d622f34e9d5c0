#!/bin/bash
# top-k parity tests, then c4 top-k at the default blocking and capped at G = 4 (1M users each)
set -e
TAG=${1:-tk}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "topk or transform or c4_scale" --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
timeout -k 10 400 python -u bench.py --steps 2 --no-cpu > gpurun_out/bench_c4_$TAG.json 2> gpurun_out/bench_c4_$TAG.err
timeout -k 10 200 python -u bench.py --config c2 --steps 3 --no-cpu --topk-users 1000000 > gpurun_out/bench_c4g4_$TAG.json 2> gpurun_out/bench_c4g4_$TAG.err
echo all-ok
