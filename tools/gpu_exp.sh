#!/bin/bash
# experiments: c5 NNLS iteration statistics; c4 split-K chunk length sweep
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu --topk-users 0 > gpurun_out/bench_c5_it.json 2> gpurun_out/bench_c5_it.err
for CH in 2048 4096 16384; do
  ALBEDO_SPLIT_CHUNK=$CH timeout -k 10 200 python -u bench.py --no-cpu --topk-users 0 > gpurun_out/bench_c4_ch$CH.json 2> gpurun_out/bench_c4_ch$CH.err
done
timeout -k 10 200 python -u bench.py --no-cpu --topk-users 0 > gpurun_out/bench_c4_ch8192.json 2> gpurun_out/bench_c4_ch8192.err
echo all-ok
