#!/bin/bash
# Short variable-length keys hashed with and without a byte count (AUTO): what the unsized
# device-resident entry point gives up when k_span_pp's 20-KiB window holds a short span.
set -e
o=${1:-gpurun_out/r3n}; mkdir -p $o
for spec in "8 64" "8 128" "8 256" "64 192"; do
  set -- $spec
  for sz in "" "--sized"; do
    echo "U[$1,$2] ${sz:-unsized}" >> $o/ab_unsized_short.txt
    timeout -k 10 120 python tools/ab.py --variant base= --workload var --var-lo $1 --var-hi $2 --n 20000000 \
      $sz --rounds 4 2>/dev/null | grep base >> $o/ab_unsized_short.txt
  done
done
cat $o/ab_unsized_short.txt
