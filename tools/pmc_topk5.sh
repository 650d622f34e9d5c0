#!/bin/bash
# SQ counter passes over the c4 top-30 scan (all 20M users after 25 sweeps), one rocprofv3 run per
# pass, every kernel collected (the scan's rows are picked by tools/sqsum.py).  usage: tools/pmc_topk5.sh <tag>
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_topk5_${1:-a}
mkdir -p $OUT
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $P --output-format csv -d $OUT/sq$i -o run -- python3 -u bench.py --steps 1 --warmup 24 --no-cpu > $OUT/sq$i.json 2> $OUT/sq$i.err
  echo "pass $i done"
done
