#!/bin/bash
# Config D's block loop taken apart: the tree against a build whose LDS block loop skips the k1/k2 mixes
# (chain only) and one that skips the h1/h2 chain (mixes only); both give wrong hashes (unchecked): what a
# split into balanced mixes + per-key chains could win at most.
set -e
o=${1:-gpurun_out/r3b}; mkdir -p $o
for spec in "8 512" "260 260"; do
  set -- $spec
  echo "U[$1,$2] sized" >> $o/ab_bounds.txt
  timeout -k 10 150 python tools/ab.py --variant tree= --variant chain=@tools/_ab/lib_chain.so --variant mix=@tools/_ab/lib_mix.so \
    --unchecked chain --unchecked mix --workload var --var-lo $1 --var-hi $2 --n 25000000 --sized --rounds 8 2>/dev/null \
    | grep -v amdgpu.ids >> $o/ab_bounds.txt
done
cat $o/ab_bounds.txt
