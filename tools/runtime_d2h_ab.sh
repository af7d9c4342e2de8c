#!/bin/bash
# Round 5: the host-inclusive lines with the caller's pageable keys handed to the
# runtime's pageable copy with the records back by the runtime's pageable D2H (SHF_HB_RUNTIME_D2H=1) and
# copied out of the slot on the copy workers (=0), alternating, three times each.
# (The SHF_HB_RUNTIME_D2H variant it measured lost and is not in the library: git history,
# profiles/r5/runtime_copy/ab_runtime_d2h/.)
set -u
o=gpurun_out/$1; mkdir -p $o
for r in 1 2 3; do
  for v in 1 0; do
    SHF_HB_RUNTIME_D2H=$v timeout -k 10 300 python bench.py --only fixed16 --no-cpu --traffic off > $o/b_${v}_$r.json 2> $o/b_${v}_$r.err || exit 1
    python3 -c "import json; d=json.loads(open('$o/b_${v}_$r.json').read().strip().splitlines()[-1])['host_inclusive']; print('runtime_d2h=$v', {k: round(x/1e9,3) for k,x in d.items() if k!='verified'}, d['verified'])"
  done
done
