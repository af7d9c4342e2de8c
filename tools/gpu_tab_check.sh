#!/bin/bash
# f4 on one GPU box: the tab-copy parity tests, then the in-tree build against
# prebuilt variants (build/ab/lib_<name>.so) on the bench's tab-part batch.
#   tools/gpu_tab_check.sh OUTDIR "name1 name2 ..."
set -u
out=$1; names=${2:-}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_tab.py -x -v --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -3 $out/pytest.log
vs="--variant new="
for nm in $names; do vs="$vs --variant $nm=@build/ab/lib_$nm.so"; done
timeout -k 10 300 python tools/ab.py --workload tab --n 1024 --rounds 5 --reps 5 $vs > $out/ab.txt 2>&1 || { tail -5 $out/ab.txt; exit 2; }
grep median $out/ab.txt
