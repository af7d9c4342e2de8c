#!/bin/bash
# Historical: the sorted span kernel lost and was removed (profiles/r1/ab_sort/);
# rerunning needs its source from git history (commit 1d01bbc).
# Sorted span kernel (SHFHB_SPAN_SORT_W = 2 or 4 waves per workgroup, keys hashed
# in block-count order; sort2asm adds SHFHB_ASM_MIX=1) against k_span: kernel 4
# in every variant, ~6.5 GB of variable-length keys U[lo, hi] per distribution.
#   python tools/ab.py --prebuild build/ab --variant sort2=-DSHFHB_SPAN_SORT_W=2 \
#       --variant sort4=-DSHFHB_SPAN_SORT_W=4 --variant "sort2asm=-DSHFHB_SPAN_SORT_W=2 -DSHFHB_ASM_MIX=1"
#   tools/gpu_sort_ab.sh OUTDIR
set -u
out=$1; mkdir -p $out
V="--variant base= --variant sort2=@build/ab/lib_sort2.so --variant sort4=@build/ab/lib_sort4.so"
V="$V --variant sort2asm=@build/ab/lib_sort2asm.so"
for d in 8:512 260:260 8:128 64:192 8:256 8:1024; do
  lo=${d%:*}; hi=${d#*:}
  n=$(( 13000000000 / (lo + hi) ))
  timeout -k 10 200 python tools/ab.py --workload var --var-lo $lo --var-hi $hi --n $n --kernel 4 --rounds 5 --reps 5 $V \
    > $out/var_${lo}_${hi}.txt 2>&1
  rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc=$rc at U[$lo,$hi]"; exit $rc; fi
done
echo ok
