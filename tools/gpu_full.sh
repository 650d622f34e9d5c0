#!/bin/bash
# Full GPU test suite (multi-rank first), then the c4 and c2 benches
set -e
TAG=${1:-x}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_multi_rank.py -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/gpu_mr_$TAG.log 2>&1
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/gpu_tests_$TAG.log 2>&1
timeout -k 10 400 python -u bench.py --no-cpu --topk-users 0 --steps 2 > gpurun_out/bench_c4_$TAG.json 2> gpurun_out/bench_c4_$TAG.err
echo all-ok
