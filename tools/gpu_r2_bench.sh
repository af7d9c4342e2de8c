#!/bin/bash
# The default bench line on one GPU box (+ its stderr).
#   tools/gpu_r2_bench.sh OUTDIR [bench args...]
set -u
out=$1; shift; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python bench.py "$@" > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail $out/bench.err; exit 3; }
cat $out/bench.err; cat $out/bench.json
