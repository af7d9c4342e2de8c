#!/bin/bash
# k_tiled round size (8 vs 16 pieces per key per round) against k_generic.
out=$1; mkdir -p $out
for L in 144 192 256 384 512; do
  n=$((6400000000 / (L + 16)))
  for R in 8 16; do
    SHF_HB_TILED_ROUND=$R timeout -k 10 120 python tools/ab.py --variant base= --workload fixedL --key-len $L --n $n --kernel 2 --rounds 3 > $out/L${L}_tiledR$R.txt 2>&1 || exit 1
  done
  timeout -k 10 120 python tools/ab.py --variant base= --workload fixedL --key-len $L --n $n --kernel 3 --rounds 3 > $out/L${L}_generic.txt 2>&1 || exit 1
done
