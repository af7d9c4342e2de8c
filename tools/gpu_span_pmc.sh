#!/bin/bash
# SQ counters of k_span builds (tools/ab.py, one variant per profiled process)
# per length distribution: where the waves' cycles go.
#   VARS="base pku" COUNTERS="..." DISTS="8:512" tools/gpu_span_pmc.sh OUTDIR
set -u
VARS=${VARS:-"base pku"}
COUNTERS=${COUNTERS:-"SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE"}
out=$1; mkdir -p $out
export TMPDIR=/tmp
for d in ${DISTS:-8:512 260:260}; do
  lo=${d%:*}; hi=${d#*:}
  n=$(( 13000000000 / (lo + hi) ))
  for v in $VARS; do
    if [ "$v" = base ]; then spec="base="; else spec="$v=@build/ab/lib_$v.so"; fi
    timeout -s KILL 120 rocprofv3 --pmc $COUNTERS \
      --output-format csv -d $out/pmc_${v}_${lo}_${hi} -o pmc -- python3 tools/ab.py --workload var --var-lo $lo --var-hi $hi --n $n \
      --kernel 0 --sized --rounds 1 --reps 2 --variant $spec > $out/pmc_${v}_${lo}_${hi}.log 2>&1 || { echo "pmc failed $v $d"; tail -5 $out/pmc_${v}_${lo}_${hi}.log; exit 1; }
    python3 tools/pmc_summary.py $out/pmc_${v}_${lo}_${hi} k_span > $out/summary_${v}_${lo}_${hi}.txt
    echo "== $v U[$lo,$hi]"; cat $out/summary_${v}_${lo}_${hi}.txt
  done
done
