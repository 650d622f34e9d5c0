#!/bin/bash
# Profile one bench config: rocprofv3 kernel trace + stats (2 timed sweeps), then separate
# FETCH_SIZE / WRITE_SIZE PMC passes over exactly one sweep -> HBM traffic per kernel.
# usage: tools/prof.sh <config> <tag>
set -e
CFG=${1:-c4}; TAG=${2:-r01}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_${CFG}_${TAG}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 -u bench.py --config $CFG --steps 2 --warmup 1 --no-cpu --topk-users 0 > $OUT/bench.json 2> $OUT/bench.err
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- \
  python3 -u bench.py --config $CFG --steps 1 --warmup 0 --no-cpu --topk-users 0 > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- \
  python3 -u bench.py --config $CFG --steps 1 --warmup 0 --no-cpu --topk-users 0 > $OUT/pmc_write.json 2> $OUT/pmc_write.err
python3 tools/traffic.py $OUT $CFG $OUT/pmc_traffic_${CFG}.json > /dev/null
echo prof done
