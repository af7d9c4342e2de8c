#!/bin/bash
# L2 hit rate and fabric requests of the f4 tab copy (tools/ab.py --workload tab),
# one rocprofv3 --pmc pass per counter group.
#   tools/gpu_tab_pmc.sh OUTDIR
set -u
out=$1; mkdir -p $out
export TMPDIR=/tmp
i=0
for grp in "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $out/p$i -o pmc -- python3 tools/ab.py --workload tab \
    --n 1024 --rounds 1 --reps 2 --warmup-s 0 --variant base= > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $out/p$i.log; exit 1; }
  python3 tools/pmc_summary.py $out/p$i k_tab_split
done
