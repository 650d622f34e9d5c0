#!/bin/bash
# Round artefacts: c4 profile (trace + traffic + SQ), default bench (c4, CPU baseline), c2, c5
set -e
TAG=${1:-r02}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash tools/prof.sh c4 $TAG 16384
python3 tools/sqsum.py gpurun_out/prof_c4_$TAG gpurun_out/prof_c4_$TAG/sq_summary.json
timeout -k 10 400 python -u bench.py > gpurun_out/bench_c4_$TAG.json 2> gpurun_out/bench_c4_$TAG.err
timeout -k 10 200 python -u bench.py --config c2 --steps 5 > gpurun_out/bench_c2_$TAG.json 2> gpurun_out/bench_c2_$TAG.err
timeout -k 10 300 python -u bench.py --config c5 --steps 2 --no-cpu --topk-users 0 > gpurun_out/bench_c5_$TAG.json 2> gpurun_out/bench_c5_$TAG.err
echo all-ok
