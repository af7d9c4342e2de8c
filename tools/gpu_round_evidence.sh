#!/bin/bash
# Round evidence on one GPU box: gpu tests, smoke, the driver's bench command,
# the per-(kernel, grid) kernel-trace profile and the PMC passes.
#   tools/gpu_round_evidence.sh OUTDIR
set -u
out=$1; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed"; exit 2; }
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --detail-out $out/bench_detail.json > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail $out/bench.err; exit 3; }
wc -c $out/bench.json
grep "\[bench\]" $out/bench.err | cut -c1-120
timeout -k 10 900 tools/profile_round.sh $out/prof > $out/profile.log 2>&1 || { echo "profile failed"; tail $out/profile.log; exit 4; }
cp $out/prof/rocprof_kernel_summary.md $out/prof/pmc_summary.txt $out/ 2>/dev/null
echo evidence ok
