#!/bin/bash
# Round 5: 16 threads sharing the staging pool (tools/diag_threads.py) under a few pool shapes.
set -u
o=gpurun_out/$1; mkdir -p $o
SHF_HB_TRACE=1 timeout -k 10 120 python -u tools/diag_threads.py --threads 16 > $o/t16_default.json 2> $o/t16_default.err || exit 1
cat $o/t16_default.json
for cfg in "SHF_HB_POOL_MB=128" "SHF_HB_COPY_THREADS=4" "SHF_HB_COPY_THREADS=2" "SHF_HB_STAGE_MB=4" "SHF_HB_POOL_MB=128 SHF_HB_COPY_THREADS=4"; do
  env $cfg timeout -k 10 120 python -u tools/diag_threads.py --threads 16 > $o/t16_$(echo $cfg | tr ' =' '__').json || exit 1
  cat $o/t16_$(echo $cfg | tr ' =' '__').json
done
timeout -k 10 120 python -u tools/diag_threads.py --threads 1 > $o/t1.json && cat $o/t1.json
timeout -k 10 120 python -u tools/diag_threads.py --threads 4 > $o/t4.json && cat $o/t4.json
