#!/bin/bash
# Round-2 GPU check: the new robustness / multi-rank tests first, then the whole
# -m gpu suite, smoke, and the default bench line.
#   tools/gpu_r2_check.sh OUTDIR
set -u
out=$1; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_robustness.py tests/test_gpu_bench.py -x -v --timeout 300 --timeout-method thread > $out/pytest_new.log 2>&1 || { echo "new tests failed"; tail -40 $out/pytest_new.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $out/pytest_gpu.log; exit 1; }
tail -3 $out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed"; exit 2; }
timeout -k 10 900 python bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail $out/bench.err; exit 3; }
cat $out/bench.err
echo check ok
