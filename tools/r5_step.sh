#!/bin/bash
# Round-5 GPU step: the GPU test suite (optionally a -k filter in $K), then the
# pageable-registration repro (tools/pageable_register_repro.sh). Stops at a
# fault, abort or timeout; a plain test failure (rc 1) still runs the repro.
set -o pipefail
mkdir -p gpurun_out/r5
if [ -n "$K" ]; then kflag=(-k "$K"); else kflag=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread "${kflag[@]}" \
  > gpurun_out/r5/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -4 gpurun_out/r5/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
[ -n "$NO_REPRO" ] && exit $rc
./tools/pageable_register_repro.sh
