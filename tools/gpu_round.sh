#!/bin/bash
# One GPU call: parity suite, then the default bench (c4) and c2, each step under its own limit.
# usage: tools/gpu_round.sh <tag>
set -e
TAG=${1:-r01}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_c4_$TAG.json 2> gpurun_out/bench_c4_$TAG.err
timeout -k 10 200 python -u bench.py --config c2 --steps 5 > gpurun_out/bench_c2_$TAG.json 2> gpurun_out/bench_c2_$TAG.err
echo all-ok
