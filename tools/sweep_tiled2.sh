#!/bin/bash
# Non-multiple-of-128 lengths: k_tiled (round 4/8/16 pieces) against k_span and k_generic.
out=$1; mkdir -p $out
for L in 144 160 176 208 240 320 448; do
  n=$((6400000000 / (L + 16)))
  for R in 4 8 16; do
    SHF_HB_TILED_ROUND=$R timeout -k 10 120 python tools/ab.py --variant base= --workload fixedL --key-len $L --n $n --kernel 2 --rounds 3 > $out/L${L}_tiledR$R.txt 2>&1 || exit 1
  done
  for K in 3 4; do
    timeout -k 10 120 python tools/ab.py --variant base= --workload fixedL --key-len $L --n $n --kernel $K --rounds 3 > $out/L${L}_k$K.txt 2>&1 || exit 1
  done
done
