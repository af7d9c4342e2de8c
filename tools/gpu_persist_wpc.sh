#!/bin/bash
# k_span_p grid size (waves per CU) against k_span, U[8,512] and all-260 B keys.
set -u
out=$1; mkdir -p $out
for d in 8:512 260:260; do
  lo=${d%:*}; hi=${d#*:}
  n=$(( 13000000000 / (lo + hi) ))
  timeout -k 10 200 python tools/ab.py --workload var --var-lo $lo --var-hi $hi --n $n --kernel 0 --sized --rounds 5 --reps 5 \
    --variant base= --variant p8=@build/ab/lib_p8.so --variant p7=@build/ab/lib_p7.so --variant p6=@build/ab/lib_p6.so \
    --variant p4=@build/ab/lib_p4.so > $out/var_${lo}_${hi}.txt 2>&1 || { echo "fail $d"; tail -5 $out/var_${lo}_${hi}.txt; exit 1; }
  echo "U[$lo,$hi]"; grep median $out/var_${lo}_${hi}.txt
done
