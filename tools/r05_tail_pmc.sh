#!/bin/bash
# usage: tools/r05_tail_pmc.sh <outdir> -- SQ / TCC counter passes over the bench step (eager, 2 steps), summarised
# per kernel (tools/pmc_summary.py): where the packed module tail and the prologue spend their cycles
O=${1:-gpurun_out/r05_tailpmc}
mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES"
P2="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
P3="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
n=0
for P in "$P1" "$P2" "$P3"; do
  n=$((n+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $O/p$n -o p -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-cfg5 --no-peaks --no-graph > $O/p$n.log 2>&1 || { echo "pass $n failed"; exit 1; }
done
python tools/pmc_summary.py $O/p*/p_counter_collection.csv > $O/summary.txt
rm -rf $O/p1 $O/p2 $O/p3
