#!/bin/bash
# f4: the tab GPU tests, then an interleaved A/B of tab-copy builds: tools/gpu_tab_ab.sh OUTDIR "names"
set -u
out=$1; names=$2; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_tab.py -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_tab.log 2>&1 || { tail -30 $out/pytest_tab.log; exit 1; }
tail -2 $out/pytest_tab.log
vs="--variant base="
for nm in $names; do vs="$vs --variant $nm=@build/ab/lib_$nm.so"; done
timeout -k 10 300 python tools/ab.py --workload tab --n 1024 --rounds 10 --reps 5 $vs > $out/tab.txt 2>&1 || { tail -5 $out/tab.txt; exit 2; }
grep median $out/tab.txt
