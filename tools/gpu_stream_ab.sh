#!/bin/bash
# k_vstream (6) against k_span (4) / k_vround (5) / k_generic (3), and its
# chunk-size / occupancy variants (prebuilt with tools/ab.py --prebuild build/ab).
#   tools/gpu_stream_ab.sh OUTDIR
set -u
out=$1; mkdir -p $out
n=25000000
timeout -k 10 240 python tools/ab.py --workload var --n $n --kernel 6 --rounds 5 --variant base= \
  --variant c256=@build/ab/lib_c256.so --variant c512=@build/ab/lib_c512.so --variant c2048=@build/ab/lib_c2048.so \
  --variant w4=@build/ab/lib_w4.so > $out/stream_variants_U8_512.txt 2>&1 || exit 1
for r in "8 512" "8 64" "8 128" "8 256" "64 192" "260 260" "8 2048"; do
  set -- $r
  n=$((13000000000 / ($1 + $2 + 48)))
  for K in 6 4 5; do
    timeout -k 10 200 python tools/ab.py --variant base= --workload var --var-lo $1 --var-hi $2 --n $n --kernel $K --rounds 3 > $out/U$1_$2_k$K.txt 2>&1 || exit 2
  done
done
echo ab ok
