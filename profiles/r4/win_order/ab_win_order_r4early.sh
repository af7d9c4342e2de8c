#!/bin/bash
# window order: tree build against the first version (tools/_ab/lib_wo7.so), bench line each, then rocprof of the tree
set -e
o=gpurun_out/wo3; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --only winorder --no-cpu --no-host-inclusive --traffic off > $o/tree.json 2> $o/tree.err
grep "\[bench\]" $o/tree.err
cp sharedhashfile_amd/libshf_hash_batch.so $o/tree.so
cp tools/_ab/lib_wo7.so sharedhashfile_amd/libshf_hash_batch.so
timeout -k 10 200 python bench.py --only winorder --no-cpu --no-host-inclusive --traffic off > $o/prev.json 2> $o/prev.err || true
grep "\[bench\]" $o/prev.err || true
cp $o/tree.so sharedhashfile_amd/libshf_hash_batch.so
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o kt -- python3 bench.py --only winorder --no-cpu --no-host-inclusive --traffic off --steps 20 --repeats 1 > $o/prof.log 2>&1
python3 tools/rocprof_summary.py $o/prof > $o/rocprof_summary.md
grep -E "k_wo" $o/rocprof_summary.md
timeout -k 10 300 tools/pmc_run.sh $o/pmc --only winorder --no-cpu --no-host-inclusive --traffic off --steps 10 --repeats 1 --no-verify > $o/pmc.log 2>&1
python3 tools/pmc_summary.py $o/pmc k_wo > $o/pmc_summary.txt
cat $o/pmc_summary.txt
