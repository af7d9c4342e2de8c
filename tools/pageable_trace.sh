#!/bin/bash
# pageable staged host path: per-repeat split from the library's SHF_HB_TRACE lines
#   tools/pageable_trace.sh OUTNAME   (on the GPU box; results under gpurun_out/OUTNAME)
export TMPDIR=/tmp
o=gpurun_out/${1:-r4k}; mkdir -p $o
SHF_HB_TRACE=1 timeout -k 10 200 python3 tools/diag_pageable_staged.py --repeats 30 --trace-file $o/ps.err > $o/pageable_staged.json 2> $o/ps.err
python3 -c "
import json; d=json.load(open('$o/pageable_staged.json')); print(d['summary'])
for r in d['repeats']: print(r)
" | head -40
