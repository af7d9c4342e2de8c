#!/bin/bash
# Host-inclusive lines, the library default against an explicit pipeline shape, alternated on one box.
set -e
o=gpurun_out/$1; mkdir -p $o
export TMPDIR=/tmp
show='import json,sys; d=json.load(open(sys.argv[1]))["host_inclusive"]; print(sys.argv[2], {k: (round(v["value"]/1e9,3), round(v["value_min"]/1e9,3), round(v["value_max"]/1e9,3)) for k, v in d.items() if isinstance(v, dict)})'
for r in 1 2 3; do
  timeout -k 10 300 python3 bench.py --only fixed16 --no-cpu --traffic off --detail-out $o/def_$r.detail.json > $o/def_$r.json 2> $o/def_$r.err
  python3 -c "$show" $o/def_$r.detail.json default
  SHF_HB_STAGE_MB=32 SHF_HB_SLOTS=3 timeout -k 10 300 python3 bench.py --only fixed16 --no-cpu --traffic off --detail-out $o/old_$r.detail.json > $o/old_$r.json 2> $o/old_$r.err
  python3 -c "$show" $o/old_$r.detail.json 32x3
done
