#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_c5_rows.py -x -v -s --timeout 480 --timeout-method thread -m gpu > gpurun_out/c5rows_batch.log 2>&1
ALBEDO_NNLS_BATCH=0 timeout -k 10 500 python -u -m pytest tests/test_gpu_c5_rows.py -x -v -s --timeout 480 --timeout-method thread -m gpu > gpurun_out/c5rows_nobatch.log 2>&1
timeout -k 10 300 python -u bench.py --config c5 --steps 2 --no-cpu --topk-users 0 > gpurun_out/bench_c5_nb2.json 2> gpurun_out/bench_c5_nb2.err
ALBEDO_NNLS_BATCH=0 timeout -k 10 300 python -u bench.py --config c5 --steps 2 --no-cpu --topk-users 0 > gpurun_out/bench_c5_nb0.json 2> gpurun_out/bench_c5_nb0.err
echo all-ok
