#!/bin/bash
# Round-end check: GPU parity suite, smoke(), default c4 bench, c2 and c5 benches, each under its own limit.
set -e
TAG=${1:-fin}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/bench_c4_$TAG.json 2> gpurun_out/bench_c4_$TAG.err
timeout -k 10 200 python -u bench.py --config c2 --no-cpu > gpurun_out/bench_c2_$TAG.json 2> gpurun_out/bench_c2_$TAG.err
timeout -k 10 300 python -u bench.py --config c5 --steps 2 --no-cpu --topk-users 0 > gpurun_out/bench_c5_$TAG.json 2> gpurun_out/bench_c5_$TAG.err
echo all-ok
