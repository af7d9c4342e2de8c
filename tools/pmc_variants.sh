#!/bin/bash
# PMC passes of config D's kernel for several prebuilt library variants (the in-tree
# library replaced by each in turn, in this scratch copy of the tree):
#   tools/pmc_variants.sh OUTDIR lib_a.so lib_b.so ...
set -u
out=$1; shift
mkdir -p "$out"
lib=sharedhashfile_amd/libshf_hash_batch.so
cp $lib $out/orig.so
for v in "$@"; do
  name=$(basename $v .so)
  cp $v $lib
  timeout -k 10 300 tools/pmc_run.sh "$out/$name" --only var --keysvar 10000000 --steps 10 --warmup 2 --repeats 1 \
    --warmup-min-s 0 --no-cpu --no-verify --no-host-inclusive --traffic off > "$out/$name.log" 2>&1 || { echo "$name failed"; cp $out/orig.so $lib; exit 1; }
  python3 tools/pmc_summary.py "$out/$name" k_span_pp > "$out/$name.txt"
  echo "== $name"; cat "$out/$name.txt"
done
cp $out/orig.so $lib
