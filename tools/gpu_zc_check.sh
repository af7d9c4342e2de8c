#!/bin/bash
# Zero-copy host path: its GPU tests, then the probe (library staged vs zero copy per key length).
set -u
mkdir -p gpurun_out/zc
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "host" > gpurun_out/zc/pytest.log 2>&1 || { tail -30 gpurun_out/zc/pytest.log; exit 1; }
tail -3 gpurun_out/zc/pytest.log
timeout -k 10 240 python tools/host_zero_copy_probe.py > gpurun_out/zc/probe3.txt 2>&1; rc=$?
cat gpurun_out/zc/probe3.txt; exit $rc
