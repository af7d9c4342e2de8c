#!/bin/bash
# Round 5: the staging pool's shape for 10M x 16-B pageable calls
# (tools/diag_pageable_staged.py, 10 repeats each): slot size SHF_HB_STAGE_MB
# x slots per call SHF_HB_SLOTS x host copy threads SHF_HB_COPY_THREADS x
# streaming (non-temporal) staging copies SHF_HB_COPY_NT, twice.
#   tools/pool_sweep.sh OUTNAME
set -u
o=gpurun_out/$1; mkdir -p $o
for r in 1 2; do
for cfg in "16 4 8 1" "16 4 8 0" "16 4 12 1" "16 4 16 1" "8 4 8 1" "32 4 8 1" "32 4 12 1" "16 3 8 1" "16 4 16 0"; do
  set -- $cfg
  timeout -k 10 200 python -u tools/diag_pageable_staged.py --repeats 10 --env SHF_HB_STAGE_MB=$1 --env SHF_HB_SLOTS=$2 \
    --env SHF_HB_COPY_THREADS=$3 --env SHF_HB_COPY_NT=$4 --env SHF_HB_POOL_MB=256 > $o/s_${1}_${2}_${3}_${4}_$r.json || exit 1
  python3 -c "import json; d=json.load(open('$o/s_${1}_${2}_${3}_${4}_$r.json'))['summary']; print('stage $1 MiB slots $2 threads $3 nt $4:', d['median'], d['min'], d['max'])"
done
done
