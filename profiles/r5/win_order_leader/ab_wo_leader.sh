#!/bin/bash
# Round 5, VERDICT r4 item 4: the window order's ranking with only each peer
# group's lowest lane reading and writing the per-wave count (base broadcast by
# ds_bpermute; tools/_ab/lead.so, built on the CPU host from a patched copy of
# csrc/win_rank.h) against the tree. Timing A/B (alternating, twice) of the
# winorder and hashwin16 lines, then one LDS-counter pass of each.
set -u
o=gpurun_out/$1; mkdir -p $o
export TMPDIR=/tmp
cp sharedhashfile_amd/libshf_hash_batch.so $o/tree.so
B="python3 bench.py --only winorder,hashwin16 --no-cpu --no-host-inclusive --traffic off"
for r in 1 2; do
  cp $o/tree.so sharedhashfile_amd/libshf_hash_batch.so
  timeout -k 10 200 $B > $o/tree$r.json 2> $o/tree$r.err || exit $?
  echo "tree: $(grep '\[bench\]' $o/tree$r.err | tr '\n' ' ')"
  cp tools/_ab/lead.so sharedhashfile_amd/libshf_hash_batch.so
  timeout -k 10 200 $B > $o/lead$r.json 2> $o/lead$r.err || exit $?
  echo "lead: $(grep '\[bench\]' $o/lead$r.err | tr '\n' ' ')"
done
for v in tree lead; do
  if [ $v = tree ]; then cp $o/tree.so sharedhashfile_amd/libshf_hash_batch.so; else cp tools/_ab/lead.so sharedhashfile_amd/libshf_hash_batch.so; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES --output-format csv \
    -d $o/pmc_$v -o pmc -- python3 bench.py --only winorder,hashwin16 --no-cpu --no-host-inclusive --traffic off --steps 5 --repeats 1 \
    > $o/pmc_$v.log 2>&1 || { echo "pmc $v failed"; cp $o/tree.so sharedhashfile_amd/libshf_hash_batch.so; exit 1; }
done
cp $o/tree.so sharedhashfile_amd/libshf_hash_batch.so
echo ab ok
