#!/bin/bash
# Round-5 GPU step: the GPU test suite (optionally a -k filter in $K; skipped
# with NO_TESTS=1), then with BENCH=1 the driver's bench command, with REPRO=1
# the pageable-registration repro. Stops at a fault, abort or timeout; a
# plain test failure (rc 1) still runs the later steps.
set -o pipefail
out=gpurun_out/r5${TAG:+_$TAG}
mkdir -p $out
rc=0
if [ -z "$NO_TESTS" ]; then
  if [ -n "$K" ]; then kflag=(-k "$K"); else kflag=(); fi
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 240 --timeout-method thread "${kflag[@]}" \
    > $out/pytest_gpu.log 2>&1
  rc=$?
  echo "pytest rc=$rc"
  tail -3 $out/pytest_gpu.log
  [ $rc -le 1 ] || exit $rc
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err
  b=$?
  echo "bench rc=$b"
  tail -c 600 $out/bench.json
  [ $b -eq 0 ] || exit $b
fi
if [ -n "$REPRO" ]; then
  ./tools/pageable_register_repro.sh || exit $?
fi
exit $rc
