#!/bin/bash
# Round evidence on one GPU box: gpu tests, smoke, the default bench line, the
# kernel-trace profile of the bench command and the PMC passes.
#   tools/gpu_round_evidence.sh OUTDIR
set -u
out=$1; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $out/pytest_gpu.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed"; exit 2; }
timeout -k 10 600 python bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail $out/bench.err; exit 3; }
cat $out/bench.json
tools/profile_round.sh $out/prof || { echo "profile failed"; exit 4; }
echo evidence ok
