#!/bin/bash
# Round 5, VERDICT r4 item 3: the row pre-probe split in two launches (pass 1
# hashes and resolves the compact map into a 16-B ticket per key, written into
# the probe output; pass 2 reads the ticket, gathers the row and overwrites
# the ticket with the record) -- tools/_ab/split.so with SHF_HB_PROBE_SPLIT=1,
# built on the CPU host from a patched copy of csrc/kernels.hip -- against the
# tree's fused kernel. Alternating, three times each, with the ceilings.
set -u
o=gpurun_out/$1; mkdir -p $o
cp sharedhashfile_amd/libshf_hash_batch.so $o/tree.so
B="python3 bench.py --only probe16,probe16_hbm,ceil_probe_rows,ceil_probe_rows_hbm --no-cpu --no-host-inclusive --traffic off"
for r in 1 2 3; do
  cp $o/tree.so sharedhashfile_amd/libshf_hash_batch.so
  timeout -k 10 300 $B > $o/tree$r.json 2> $o/tree$r.err || { cp $o/tree.so sharedhashfile_amd/libshf_hash_batch.so; exit 1; }
  echo "tree: $(grep '\[bench\]' $o/tree$r.err | tr '\n' ' ')"
  cp tools/_ab/split.so sharedhashfile_amd/libshf_hash_batch.so
  SHF_HB_PROBE_SPLIT=1 timeout -k 10 300 $B > $o/split$r.json 2> $o/split$r.err || { cp $o/tree.so sharedhashfile_amd/libshf_hash_batch.so; exit 1; }
  echo "split: $(grep '\[bench\]' $o/split$r.err | tr '\n' ' ')"
done
cp $o/tree.so sharedhashfile_amd/libshf_hash_batch.so
grep -h '"verified"' $o/split*.json | head -c 0
echo ab ok
