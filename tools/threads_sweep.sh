#!/bin/bash
# Round 5: k threads sharing the staging pool (tools/diag_threads.py) under a few pool shapes.
set -u
o=gpurun_out/$1; mkdir -p $o
for k in 16 1 4; do
  timeout -k 10 120 python -u tools/diag_threads.py --threads $k > $o/t${k}.json || exit 1
  cat $o/t${k}.json
done
for cfg in "SHF_HB_POOL_MB=128" "SHF_HB_COPY_THREADS=4"; do
  env $cfg timeout -k 10 120 python -u tools/diag_threads.py --threads 16 > $o/t16_$(echo $cfg | tr ' =' '__').json || exit 1
  cat $o/t16_$(echo $cfg | tr ' =' '__').json
done
