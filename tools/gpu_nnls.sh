#!/bin/bash
# NNLS check: parity tests of both NNLS kernels, the c5 full-size rows, then the c5 bench (tag $1)
set -e
TAG=${1:-nb}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_heavy_tail.py tests/test_gpu_c5_rows.py -x -v -s --timeout 300 --timeout-method thread -m gpu -k "nnls or c5 or million or inject or gram_is or albedo_protocol" > gpurun_out/nnls_tests_$TAG.log 2>&1
timeout -k 10 300 python -u bench.py --config c5 --steps 2 --no-cpu --topk-users 0 > gpurun_out/bench_c5_$TAG.json 2> gpurun_out/bench_c5_$TAG.err
echo all-ok
