#!/bin/bash
# Kernel choice per fixed key length: tiled (2) vs span (4) vs generic (3).
out=$1; mkdir -p $out
for L in 24 32 48 64 100 128 192 256; do
  for k in 2 4 3; do
    if [ $k = 2 ] && [ $((L % 16)) != 0 ]; then continue; fi
    n=$((6400000000 / (L + 16)))
    timeout -k 10 120 python tools/ab.py --variant base= --workload fixedL --key-len $L --n $n --kernel $k --rounds 3 > $out/L${L}_k$k.txt 2>&1 || exit 1
  done
done
