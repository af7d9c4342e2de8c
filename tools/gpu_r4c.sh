#!/bin/bash
# round-4 window-order iteration: the ballot scatter with phases removed (timing only)
export TMPDIR=/tmp
o=gpurun_out/${1:-r4c}; mkdir -p $o
B="timeout -k 10 200 python3 bench.py --only winorder --no-cpu --no-host-inclusive --traffic off --no-verify"
for v in 1 20 21 22 23 24 27; do
  SHF_HB_WO_SCATTER=$v $B > $o/b_$v.json 2> $o/b_$v.err; echo "scatter $v"; grep "\[bench\]" $o/b_$v.err
done
for v in 1 20 27; do
SHF_HB_WO_SCATTER=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof$v -o kt -- python3 bench.py --only winorder --no-cpu --no-host-inclusive --traffic off --no-verify --steps 20 --repeats 1 > $o/prof.log 2>&1
python3 tools/rocprof_summary.py $o/prof$v > $o/rocprof_summary$v.md; grep -E "k_wo" $o/rocprof_summary$v.md
done
timeout -k 10 200 python3 tools/diag_pageable_staged.py --repeats 20 > $o/pageable_staged.json 2> $o/pageable_staged.err; python3 -c "import json; d=json.load(open('$o/pageable_staged.json')); print(d['summary']); [print(r) for r in d['repeats'] if r['gkeys_s'] < 0.85 * d['summary']['median']]"
timeout -k 10 200 python3 tools/diag_pageable_staged.py --repeats 10 --fresh-out > $o/pageable_staged_fresh.json 2>> $o/pageable_staged.err; python3 -c "import json; d=json.load(open('$o/pageable_staged_fresh.json')); print(d['summary'])"
