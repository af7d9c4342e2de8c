#!/bin/bash
# Round-end evidence on the GPU box: kernel-trace stats of the bench command and
# PMC passes (separate runs; --pmc never mixed with tracing).
#   tools/profile_round.sh OUTDIR
set -u
out=$1; mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt" -o kt -- \
  python3 bench.py --steps 20 --warmup 3 --repeats 1 --warmup-min-s 0 --no-cpu --no-verify --no-host-inclusive --traffic off > "$out/kt_bench.json" 2> "$out/kt_bench.err" || exit 1
tools/pmc_run.sh "$out/pmc" --steps 3 --warmup 1 --repeats 1 --warmup-min-s 0 --no-cpu --no-verify --no-host-inclusive --traffic off > "$out/pmc.log" 2>&1 || exit 2
echo profile ok
