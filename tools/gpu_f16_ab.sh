#!/bin/bash
# k_fixed16 launch-shape variants and plain vs HIP-graph launches (10M and 100M keys).
set -u
out=$1; mkdir -p $out
V="--variant base= --variant kpl2=@build/ab/lib_kpl2.so --variant b128=@build/ab/lib_b128.so --variant b512=@build/ab/lib_b512.so --variant b1024=@build/ab/lib_b1024.so --variant ntst=@build/ab/lib_ntst.so"
timeout -k 10 200 python tools/ab.py --workload fixed16 --n 10000000 --kernel 1 --rounds 9 --reps 20 $V > $out/f16_10M.txt 2>&1 || exit 1
timeout -k 10 200 python tools/ab.py --workload fixed16 --n 10000000 --kernel 1 --rounds 9 --reps 20 --graph $V > $out/f16_10M_graph.txt 2>&1 || exit 2
timeout -k 10 200 python tools/ab.py --workload fixed16 --n 100000000 --kernel 1 --rounds 7 --reps 5 $V --copy-ref > $out/f16_100M.txt 2>&1 || exit 3
echo ok
