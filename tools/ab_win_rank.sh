#!/bin/bash
# Window order A/B: the tree's library against a previous build (tools/_ab/$2.so), the
# winorder + hashwin16 lines twice each, alternating; then kernel-trace stats of the tree.
set -e
o=gpurun_out/$1; mkdir -p $o
export TMPDIR=/tmp
cp sharedhashfile_amd/libshf_hash_batch.so $o/tree.so
B="python3 bench.py --only winorder,hashwin16 --no-cpu --no-host-inclusive --traffic off"
for r in 1 2; do
  cp $o/tree.so sharedhashfile_amd/libshf_hash_batch.so
  timeout -k 10 200 $B > $o/tree$r.json 2> $o/tree$r.err; echo "tree: $(grep '\[bench\]' $o/tree$r.err | tr '\n' ' ')"
  cp tools/_ab/$2.so sharedhashfile_amd/libshf_hash_batch.so
  timeout -k 10 200 $B > $o/prev$r.json 2> $o/prev$r.err; echo "prev: $(grep '\[bench\]' $o/prev$r.err | tr '\n' ' ')"
done
cp $o/tree.so sharedhashfile_amd/libshf_hash_batch.so
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$o/prof -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --only winorder,hashwin16 --no-cpu --no-host-inclusive --traffic off --steps 20 --repeats 1 > $GRAFT_REPO_ROOT/$o/prof.log 2>&1
cd $GRAFT_REPO_ROOT
python3 tools/rocprof_summary.py $o/prof > $o/rocprof_summary.md
grep -E "k_wo|k_fixed16_win" $o/rocprof_summary.md
