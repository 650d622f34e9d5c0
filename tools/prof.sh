#!/bin/bash
# Profile one bench config (round 2 layout):
#  1. rocprofv3 --kernel-trace --stats over 2 timed sweeps + a top-30 run on --topk-users users
#  2. FETCH_SIZE / WRITE_SIZE passes over exactly one sweep -> per-kernel HBM bytes (tools/traffic.py)
#  3. SQ passes (MFMA busy cycles, waits, instruction mix) over one sweep + the top-30 run
# usage: tools/prof.sh <config> <tag> [topk-users]
set -e
CFG=${1:-c4}; TAG=${2:-r02}; TK=${3:-16384}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_${CFG}_${TAG}
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 -u bench.py --config $CFG --steps 2 --warmup 1 --no-cpu --topk-users $TK > $OUT/bench.json 2> $OUT/bench.err
echo trace done
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- \
  python3 -u bench.py --config $CFG --steps 1 --warmup 0 --no-cpu --topk-users 0 > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- \
  python3 -u bench.py --config $CFG --steps 1 --warmup 0 --no-cpu --topk-users 0 > $OUT/pmc_write.json 2> $OUT/pmc_write.err
python3 tools/traffic.py $OUT $CFG $OUT/pmc_traffic_${CFG}.json > /dev/null
echo traffic done
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES" \
         "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $P --output-format csv -d $OUT/sq$i -o run -- \
    python3 -u bench.py --config $CFG --steps 1 --warmup 0 --no-cpu --topk-users $TK > $OUT/sq$i.json 2> $OUT/sq$i.err
done
echo prof done
