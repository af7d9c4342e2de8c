#!/bin/bash
# Historical: build/ab/lib_prev.so was built from commit 97e06d7's csrc
# (profiles/r1/ab_sized_small/vs_prev_*).
# Sized windows: the current rule (small windows without the round fallback,
# 4/10-KiB fetches) against the previous one (10-20 KiB, round fallback), same
# process, kernel AUTO with the byte count. build/ab/lib_prev.so = commit 97e06d7.
set -u
out=$1; mkdir -p $out
for d in 8:64 8:128 64:192 8:256 8:384 8:512; do
  lo=${d%:*}; hi=${d#*:}
  n=$(( 13000000000 / (lo + hi) ))
  timeout -k 10 200 python tools/ab.py --workload var --var-lo $lo --var-hi $hi --n $n --kernel 0 --sized --rounds 7 --reps 5 \
    --variant base= --variant prev=@build/ab/lib_prev.so > $out/var_${lo}_${hi}.txt 2>&1
  rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc=$rc at U[$lo,$hi]"; exit $rc; fi
done
echo ok
