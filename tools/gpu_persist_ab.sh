#!/bin/bash
# k_span (one tile per workgroup) vs k_span_p (persistent waves, next span in
# flight during the hash) per length distribution, kernel AUTO, ~6.5 GB.
#   tools/gpu_persist_ab.sh OUTDIR
set -u
out=$1; mkdir -p $out
for d in ${DISTS:-8:512 260:260 64:192 8:256 200:400}; do
  lo=${d%:*}; hi=${d#*:}
  n=$(( 13000000000 / (lo + hi) ))
  for sized in ${SIZED:-"" "--sized"}; do
    timeout -k 10 200 python tools/ab.py --workload var --var-lo $lo --var-hi $hi --n $n --kernel 0 $sized --rounds 5 --reps 5 \
      --variant base= --variant persist=@build/ab/lib_persist.so > $out/var_${lo}_${hi}${sized}.txt 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "fatal rc=$rc at U[$lo,$hi] $sized"; tail -5 $out/var_${lo}_${hi}${sized}.txt; exit $rc; fi
    echo "U[$lo,$hi] $sized"; cat $out/var_${lo}_${hi}${sized}.txt
  done
done
echo ok
