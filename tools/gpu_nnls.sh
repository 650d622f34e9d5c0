#!/bin/bash
# NNLS check: parity tests of both NNLS kernels, then the c5 bench (tag as $1)
set -e
TAG=${1:-nb}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -m gpu -k "nnls" > gpurun_out/nnls_tests_$TAG.log 2>&1
timeout -k 10 300 python -u bench.py --config c5 --steps 2 --no-cpu --topk-users 0 > gpurun_out/bench_c5_$TAG.json 2> gpurun_out/bench_c5_$TAG.err
echo all-ok
