#!/bin/bash
# PMC passes over the solve kernels of one bench sweep (each pass its own rocprofv3 run).
# usage: tools/pmc.sh <config> <tag> [kernel-regex]
set -e
CFG=${1:-c4}; TAG=${2:-r01}; RX=${3:-solve_}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_${CFG}_${TAG}
mkdir -p $OUT
BENCH="python -u bench.py --config $CFG --steps 1 --warmup 0 --no-cpu --topk-users 0"
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LEVEL_WAVES SQ_INSTS_VMEM_RD" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --kernel-include-regex "$RX" --output-format csv -d $OUT/p$i -o run -- $BENCH > $OUT/p$i.json 2> $OUT/p$i.err
done
echo pmc done
