#!/bin/bash
# AUTO on short and mid fixed key lengths (bytes/key = L + 16), 100M keys each, against the 16-B copy
# (--copy-ref: torch copy_ of the same byte count) -- where a fixed length sits below its ceiling.
set -e
o=${1:-gpurun_out/r3v}; mkdir -p $o
for L in 4 8 12 16 24 32 48 64; do
  echo "L=$L" >> $o/ab_fixed_lengths.txt
  timeout -k 10 120 python tools/ab.py --variant auto= --workload fixedL --key-len $L --n 100000000 --rounds 4 \
    --copy-ref 2>/dev/null | grep -v amdgpu.ids >> $o/ab_fixed_lengths.txt
done
cat $o/ab_fixed_lengths.txt
