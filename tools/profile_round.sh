#!/bin/bash
# Round evidence on the GPU box: kernel-trace stats of the bench, one rocprofv3
# pass per group of workloads (the headline alone, so its 10M-key k_fixed16
# launches are the only ones of their kernel and grid), summarised per
# (kernel, grid); then the PMC passes (separate runs; --pmc never mixed with
# tracing).
#   tools/profile_round.sh OUTDIR
set -u
out=$1; mkdir -p "$out"
export TMPDIR=/tmp
common="--steps 20 --warmup 3 --repeats 1 --warmup-min-s 0.5 --no-cpu --no-verify --no-host-inclusive --traffic off"
i=0
for only in "fixed16" "ceil_copy,ceil_copy_hot,fixed16_hot" "shard1b,ceil_copy_1b" "fixed256,ceil_read16,ceil_read16nt,ceil_read16w1" \
            "var" "probe16,ceil_gather128" "probe16_hbm,ceil_probe_rows_hbm" "tabpart,ceil_copynt,ceil_stream16u" "winorder" \
            "hashwin16" "ceil_valu_add,ceil_valu_mul"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt$i" -o kt -- \
    python3 bench.py $common --only "$only" > "$out/kt$i.json" 2> "$out/kt$i.err" || { echo "kt pass $i ($only) failed"; exit 1; }
  python3 tools/rocprof_summary.py "$out/kt$i" --label "bench.py --only $only" >> "$out/rocprof_kernel_summary.md"
  echo >> "$out/rocprof_kernel_summary.md"
done
tools/pmc_run.sh "$out/pmc" --steps 3 --warmup 1 --repeats 1 --warmup-min-s 0 --no-cpu --no-verify --no-host-inclusive --traffic off > "$out/pmc.log" 2>&1 || exit 2
python3 tools/pmc_summary.py "$out/pmc" > "$out/pmc_summary.txt"
echo profile ok
