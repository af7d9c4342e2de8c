#!/bin/bash
# Round 5: host-inclusive lines with the fixed-length pipeline's last chunk tapered (SHF_HB_TAPER=1)
# or not (0), alternating, three times each.
set -u
o=gpurun_out/$1; mkdir -p $o
for r in 1 2 3; do
  for v in 1 0; do
    SHF_HB_TAPER=$v timeout -k 10 300 python bench.py --only fixed16 --no-cpu --traffic off > $o/b_${v}_$r.json 2> $o/b_${v}_$r.err || exit 1
    python3 -c "import json; d=json.loads(open('$o/b_${v}_$r.json').read().strip().splitlines()[-1])['host_inclusive']; print('taper=$v', {k: round(x/1e9,3) for k,x in d.items() if k!='verified'}, d['verified'])"
  done
done
