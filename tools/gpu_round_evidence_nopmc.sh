#!/bin/bash
# Round evidence without the PMC passes (kernels unchanged since their last profile):
# gpu tests, smoke, the driver bench command.  tools/gpu_round_evidence_nopmc.sh [OUTDIR]
set -u
out=${1:-gpurun_out/evidence}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed"; exit 2; }
s=$(date +%s)
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --detail-out $out/bench_detail.json > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail $out/bench.err; exit 3; }
echo "bench wall s: $(( $(date +%s) - s ))" | tee $out/bench_wall.txt
wc -c $out/bench.json
echo evidence ok
