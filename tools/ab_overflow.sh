#!/bin/bash
# k_span_pp's overflow tiles (spans over the window, keys hashed without a byte count): the tree's build
# against a saved one (tools/_ab/lib_head.so), same process, several length distributions.
set -e
o=${1:-gpurun_out/r3k}; mkdir -p $o
for spec in "8 2048 0" "8 1024 0" "8 512 0" "8 512 1" "260 260 1"; do
  set -- $spec
  sz=""; [ "$3" = 1 ] && sz="--sized"
  echo "U[$1,$2] sized=$3" >> $o/ab_overflow.txt
  timeout -k 10 150 python tools/ab.py --variant head=@tools/_ab/lib_head.so --variant new= --workload var \
    --var-lo $1 --var-hi $2 --n 5000000 $sz --rounds 6 2>/dev/null | grep -E "head|new" >> $o/ab_overflow.txt
done
cat $o/ab_overflow.txt
