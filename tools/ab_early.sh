#!/bin/bash
# k_span_pp hand-over at wave 0's last LDS read (tail + fmix after the barrier) against a saved build
# (tools/_ab/lib_head.so): config D's distribution sized and unsized, all-260 B, U[64,448].
set -e
o=${1:-gpurun_out/r3x}; mkdir -p $o
for spec in "8 512 1" "8 512 0" "260 260 1" "64 448 1"; do
  set -- $spec
  sz=""; [ "$3" = 1 ] && sz="--sized"
  echo "U[$1,$2] sized=$3" >> $o/ab_early_addr.txt
  timeout -k 10 150 python tools/ab.py --variant head=@tools/_ab/lib_head.so --variant early=@tools/_ab/lib_early.so --variant addr= --workload var \
    --var-lo $1 --var-hi $2 --n 25000000 $sz --rounds 8 2>/dev/null | grep -v amdgpu.ids >> $o/ab_early_addr.txt
done
cat $o/ab_early_addr.txt
