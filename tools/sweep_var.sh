#!/bin/bash
# Variable-length kernels (k_span = 4, k_vround = 5, k_generic = 3) per length
# distribution U[lo, hi], ~6.5 GB of key bytes each.
out=$1; mkdir -p $out
for r in "8 64" "8 128" "8 256" "64 192" "8 512" "260 260" "8 2048"; do
  set -- $r
  n=$((13000000000 / ($1 + $2 + 48)))
  for K in 4 5 3; do
    timeout -k 10 200 python tools/ab.py --variant base= --workload var --var-lo $1 --var-hi $2 --n $n --kernel $K --rounds 3 > $out/U$1_$2_k$K.txt 2>&1 || exit 1
  done
done
