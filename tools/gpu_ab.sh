#!/bin/bash
# GPU call: parity suite, then c4 with the default heavy kernel and with ALBEDO_HEAVY=wg (A/B), then c2.
# usage: tools/gpu_ab.sh <tag> [skip-tests]
set -e
TAG=${1:-ab}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
fi
timeout -k 10 300 python -u bench.py --no-cpu --topk-users 0 > gpurun_out/bench_c4_$TAG.json 2> gpurun_out/bench_c4_$TAG.err
ALBEDO_HEAVY=wg timeout -k 10 300 python -u bench.py --no-cpu --topk-users 0 > gpurun_out/bench_c4wg_$TAG.json 2> gpurun_out/bench_c4wg_$TAG.err
timeout -k 10 200 python -u bench.py --config c2 --steps 5 --no-cpu --topk-users 0 > gpurun_out/bench_c2_$TAG.json 2> gpurun_out/bench_c2_$TAG.err
echo all-ok
