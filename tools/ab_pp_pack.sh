#!/bin/bash
# k_span_pp packing two tiles' spans into its window at once: the tree's build against a saved one
# (tools/_ab/lib_head.so) and optional extra variants (lib_*.so given as arguments), same process,
# sized and unsized batches.
set -e
o=gpurun_out/r3o; mkdir -p $o
extra=""; for v in "$@"; do extra="$extra --variant $(basename $v .so | sed s/lib_//)=@$v"; done
for spec in "8 64 0" "8 128 0" "8 256 0" "8 512 0" "8 512 1" "260 260 1" "8 2048 0"; do
  set -- $spec
  sz=""; [ "$3" = 1 ] && sz="--sized"
  echo "U[$1,$2] sized=$3" >> $o/ab_pp_pack.txt
  timeout -k 10 150 python tools/ab.py --variant head=@tools/_ab/lib_head.so --variant new= $extra --workload var \
    --var-lo $1 --var-hi $2 --n 10000000 $sz --rounds 6 2>/dev/null | grep -v amdgpu.ids >> $o/ab_pp_pack.txt
done
cat $o/ab_pp_pack.txt
