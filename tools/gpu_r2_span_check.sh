#!/bin/bash
# After adopting k_span_pp + unaligned LDS reads: the whole -m gpu suite, then
# the in-tree build against the previous commit's (build/ab/lib_head.so) on
# variable-length distributions and on fixed lengths that take k_span.
set -u
out=$1; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
for d in 8:512 260:260 8:128 8:256 64:192 200:400 8:1024; do
  lo=${d%:*}; hi=${d#*:}
  n=$(( 13000000000 / (lo + hi) ))
  timeout -k 10 200 python tools/ab.py --workload var --var-lo $lo --var-hi $hi --n $n --kernel 0 --sized --rounds 5 --reps 5 \
    --variant new= --variant head=@build/ab/lib_head.so > $out/var_${lo}_${hi}.txt 2>&1 || { echo "fail $d"; tail -5 $out/var_${lo}_${hi}.txt; exit 1; }
  echo "U[$lo,$hi] sized"; grep median $out/var_${lo}_${hi}.txt
done
timeout -k 10 200 python tools/ab.py --workload var --var-lo 8 --var-hi 512 --n 25000000 --kernel 0 --rounds 5 --reps 5 \
  --variant new= --variant head=@build/ab/lib_head.so > $out/var_8_512_unsized.txt 2>&1 || exit 1
echo "U[8,512] unsized"; grep median $out/var_8_512_unsized.txt
for L in 48 100 200 300; do
  timeout -k 10 200 python tools/ab.py --workload fixedL --key-len $L --n $(( 6400000000 / L )) --kernel 0 --rounds 5 --reps 5 \
    --variant new= --variant head=@build/ab/lib_head.so > $out/fixed_$L.txt 2>&1 || { echo "fail L=$L"; exit 1; }
  echo "fixed L=$L"; grep median $out/fixed_$L.txt
done
echo ok
