#!/bin/bash
# Like gpu_span_ab2.sh with more rounds (small effects): tools/gpu_span_ab3.sh OUTDIR "names" ["lo:hi ..."]
set -u
out=$1; names=$2; dists=${3:-"8:512 260:260"}
mkdir -p $out
vs="--variant base="
for nm in $names; do vs="$vs --variant $nm=@build/ab/lib_$nm.so"; done
for d in $dists; do
  lo=${d%:*}; hi=${d#*:}
  n=$(( 13000000000 / (lo + hi) ))
  timeout -k 10 300 python tools/ab.py --workload var --var-lo $lo --var-hi $hi --n $n --kernel 0 --sized --rounds 12 --reps 5 \
    $vs > $out/var_${lo}_${hi}.txt 2>&1 || { echo "fail $d"; tail -5 $out/var_${lo}_${hi}.txt; exit 1; }
  echo "U[$lo,$hi]"; grep median $out/var_${lo}_${hi}.txt
done
