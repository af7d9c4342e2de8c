#!/bin/bash
# k_span2 (7, two-phase) against k_span (4) per length distribution.
set -u
out=$1; mkdir -p $out
for r in "8 512" "260 260" "8 256" "64 192" "8 128" "8 64" "8 2048"; do
  set -- $r
  n=$((13000000000 / ($1 + $2 + 48)))
  for K in 7 4; do
    timeout -k 10 200 python tools/ab.py --variant base= --workload var --var-lo $1 --var-hi $2 --n $n --kernel $K --rounds 3 > $out/U$1_$2_k$K.txt 2>&1 || exit 2
  done
done
echo ab ok
