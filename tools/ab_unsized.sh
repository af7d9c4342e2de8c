#!/bin/bash
# Variable-length keys hashed without a byte count (the default hash_var path): AUTO against every
# variable-length kernel, for long keys (U[8,2048]) and config D's lengths. One process per run.
set -e
o=gpurun_out/r3j; mkdir -p $o
for lh in "8 2048" "8 512"; do
  set -- $lh
  for k in 0 4 5 6 3; do
    echo "U[$1,$2] unsized kernel=$k" >> $o/unsized.txt
    timeout -k 10 120 python tools/ab.py --variant base= --workload var --var-lo $1 --var-hi $2 --n 5000000 --kernel $k --rounds 4 2>/dev/null | grep base >> $o/unsized.txt
  done
  echo "U[$1,$2] sized AUTO" >> $o/unsized.txt
  timeout -k 10 120 python tools/ab.py --variant base= --workload var --var-lo $1 --var-hi $2 --n 5000000 --sized --rounds 4 2>/dev/null | grep base >> $o/unsized.txt
done
cat $o/unsized.txt
