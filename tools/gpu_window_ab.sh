#!/bin/bash
# Historical: SHFHB_SPAN_ALLOC was a one-off build flag (profiles/r1/ab_window/);
# the window is now sized per launch (kernels.hip launch_span).
# k_span LDS window per tile (SHFHB_SPAN_ALLOC bytes: 16384 -> 10 tiles per CU,
# 18176 -> 9, 20480 -> 8 (base), 23296 -> 7, 27264 -> 6) per length distribution.
#   python tools/ab.py --prebuild build/ab --variant w16=-DSHFHB_SPAN_ALLOC=16384 ...
#   tools/gpu_window_ab.sh OUTDIR
set -u
out=$1; mkdir -p $out
V="--variant base= --variant w16=@build/ab/lib_w16.so --variant w18=@build/ab/lib_w18.so"
V="$V --variant w23=@build/ab/lib_w23.so --variant w27=@build/ab/lib_w27.so"
for d in 8:512 260:260 8:256 64:192 8:1024; do
  lo=${d%:*}; hi=${d#*:}
  n=$(( 13000000000 / (lo + hi) ))
  timeout -k 10 200 python tools/ab.py --workload var --var-lo $lo --var-hi $hi --n $n --kernel 4 --rounds 5 --reps 5 $V \
    > $out/var_${lo}_${hi}.txt 2>&1
  rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc=$rc at U[$lo,$hi]"; exit $rc; fi
done
echo ok
