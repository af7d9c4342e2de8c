#!/bin/bash
# round-4 window-order iteration: phase-1 cost split (match VALU vs the count chain), timing only
export TMPDIR=/tmp
o=gpurun_out/${1:-r4c}; mkdir -p $o
B="timeout -k 10 200 python3 bench.py --only winorder --no-cpu --no-host-inclusive --traffic off --no-verify"
for v in 20 264 2128 2192 25; do
  SHF_HB_WO_SCATTER=$v $B > $o/b_$v.json 2> $o/b_$v.err; echo "scatter $v $(grep '\[bench\]' $o/b_$v.err | tr '\n' ' ')"
done
