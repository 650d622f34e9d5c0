#!/bin/bash
# One GPU call of round 2: parity suite, then the default bench (c4) and c5, each under its own limit.
# usage: tools/gpu_r02.sh <tag> [skip-tests]
set -e
TAG=${1:-r02}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
fi
timeout -k 10 400 python -u bench.py > gpurun_out/bench_c4_$TAG.json 2> gpurun_out/bench_c4_$TAG.err
timeout -k 10 300 python -u bench.py --config c5 --steps 2 --no-cpu --topk-users 0 > gpurun_out/bench_c5_$TAG.json 2> gpurun_out/bench_c5_$TAG.err
echo all-ok
