#!/bin/bash
# Variable-length batches with and without the batch byte count (the sized
# window, shf_hash_batch_var_sized_kernel_async), kernel AUTO, ~6.5 GB per
# length distribution U[lo, hi]; the round kernel alone for reference.
#   tools/gpu_sized_ab.sh OUTDIR
set -u
out=$1; mkdir -p $out
for d in 8:64 8:128 64:192 8:256 8:384 8:512 260:260 8:1024; do
  lo=${d%:*}; hi=${d#*:}
  n=$(( 13000000000 / (lo + hi) ))
  for mode in unsized sized round; do
    case $mode in
      unsized) extra="--kernel 0" ;;
      sized) extra="--kernel 0 --sized" ;;
      round) extra="--kernel 5" ;;
    esac
    timeout -k 10 200 python tools/ab.py --workload var --var-lo $lo --var-hi $hi --n $n $extra --rounds 5 --reps 5 \
      --variant $mode= > $out/${mode}_${lo}_${hi}.txt 2>&1
    rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc=$rc at U[$lo,$hi] $mode"; exit $rc; fi
  done
done
echo ok
