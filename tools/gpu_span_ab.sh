#!/bin/bash
# k_span variants (prebuilt into build/ab/lib_<name>.so) against the in-tree
# library per length distribution, kernel AUTO with the batch byte count, ~6.5 GB.
#   tools/gpu_span_ab.sh OUTDIR "name1 name2 ..." ["lo:hi lo:hi ..."]
set -u
out=$1; names=$2; dists=${3:-"8:512 260:260 8:128 8:256 200:400"}
mkdir -p $out
vs="--variant base="
for nm in $names; do vs="$vs --variant $nm=@build/ab/lib_$nm.so"; done
for d in $dists; do
  lo=${d%:*}; hi=${d#*:}
  n=$(( 13000000000 / (lo + hi) ))
  timeout -k 10 200 python tools/ab.py --workload var --var-lo $lo --var-hi $hi --n $n --kernel 0 --sized --rounds 5 --reps 5 \
    $vs > $out/var_${lo}_${hi}.txt 2>&1 || { echo "fail $d"; tail -5 $out/var_${lo}_${hi}.txt; exit 1; }
  echo "U[$lo,$hi]"; grep median $out/var_${lo}_${hi}.txt
done
