#!/bin/bash
# Bench lines under several library builds (tools/_ab/<name>.so), alternating, twice:
#   tools/ab_lines.sh OUT LINES NAME...   (the tree's library is restored at the end)
set -e
o=gpurun_out/$1; lines=$2; shift 2; mkdir -p $o
export TMPDIR=/tmp
cp sharedhashfile_amd/libshf_hash_batch.so $o/tree.so
for r in 1 2; do
  for nm in "$@"; do
    cp tools/_ab/$nm.so sharedhashfile_amd/libshf_hash_batch.so
    timeout -k 10 300 python3 bench.py --only $lines --no-cpu --no-host-inclusive --traffic off > $o/${nm}_$r.json 2> $o/${nm}_$r.err
    echo "$nm: $(grep '\[bench\]' $o/${nm}_$r.err | tr '\n' ' ')"
  done
done
cp $o/tree.so sharedhashfile_amd/libshf_hash_batch.so
