#!/bin/bash
# k_span_pp: the tree against (single) one code path for both waves' stage + hash (the barrier placed
# per wave) and (split) that path with the tile's k1/k2 mixes spread evenly over the lanes and written
# back in place, then per-key chains. Outputs compared against the tree's.
set -e
o=${1:-gpurun_out/r3s}; mkdir -p $o
for spec in "8 512 1" "260 260 1" "64 448 1" "8 512 0"; do
  set -- $spec
  sz=""; [ "$3" = 1 ] && sz="--sized"
  echo "U[$1,$2] sized=$3" >> $o/ab_split3.txt
  timeout -k 10 150 python tools/ab.py --variant tree= --variant single=@tools/_ab/lib_single.so --variant split=@tools/_ab/lib_split.so \
    --workload var --var-lo $1 --var-hi $2 --n 25000000 $sz --rounds 8 2>/dev/null | grep -v amdgpu.ids >> $o/ab_split3.txt
done
cat $o/ab_split3.txt
