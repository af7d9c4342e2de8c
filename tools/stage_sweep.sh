#!/bin/bash
# Host pipeline shape sweep: 10M x 16-B pageable calls (tools/diag_pageable_staged.py) per
# SHF_HB_STAGE_MB x SHF_HB_SLOTS, twice, then the bench's host-inclusive lines at two shapes.
set -e
o=gpurun_out/$1; mkdir -p $o
export TMPDIR=/tmp
for r in 1 2; do
for cfg in "32 3" "8 4" "8 3" "4 4" "2 4"; do
  set -- $cfg
  timeout -k 10 200 python -u tools/diag_pageable_staged.py --repeats 10 --env SHF_HB_STAGE_MB=$1 --env SHF_HB_SLOTS=$2 > $o/s_${1}_${2}_$r.json
  python3 -c "import json; d=json.load(open('$o/s_${1}_${2}_$r.json'))['summary']; print('stage $1 MiB slots $2:', d['median'], d['min'], d['max'])"
done
done
for cfg in "32 3" "8 4"; do
  set -- $cfg
  SHF_HB_STAGE_MB=$1 SHF_HB_SLOTS=$2 timeout -k 10 300 python3 bench.py --only fixed16 --no-cpu --traffic off > $o/b_${1}_${2}.json 2> $o/b_${1}_${2}.err
  python3 -c "import json; d=json.load(open('$o/b_${1}_${2}.json')); print('bench $1 MiB slots $2:', d.get('host_inclusive'))"
done
