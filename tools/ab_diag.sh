#!/bin/bash
# Kernel-trace stats of one bench line under several library builds (tools/_ab/<name>.so):
#   tools/ab_diag.sh OUT LINE NAME...   (the tree's library is restored at the end)
set -e
o=gpurun_out/$1; line=$2; shift 2; mkdir -p $o
export TMPDIR=/tmp
cp sharedhashfile_amd/libshf_hash_batch.so $o/tree.so
for nm in "$@"; do
  cp tools/_ab/$nm.so sharedhashfile_amd/libshf_hash_batch.so
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$o/p_$nm -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --only $line --no-cpu --no-host-inclusive --traffic off --no-verify --steps 20 --repeats 1 > $GRAFT_REPO_ROOT/$o/p_$nm.log 2>&1)
  python3 tools/rocprof_summary.py $o/p_$nm > $o/s_$nm.md
  echo "== $nm"; grep -E "k_wo|k_fixed16" $o/s_$nm.md
done
cp $o/tree.so sharedhashfile_amd/libshf_hash_batch.so
