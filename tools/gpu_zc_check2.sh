#!/bin/bash
set -u
mkdir -p gpurun_out/zc3
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_robustness.py -m gpu -x -v --timeout 120 --timeout-method thread -k "host" > gpurun_out/zc3/pytest.log 2>&1 || { tail -30 gpurun_out/zc3/pytest.log; exit 1; }
tail -2 gpurun_out/zc3/pytest.log
timeout -k 10 600 python bench.py > gpurun_out/zc3/bench.json 2> gpurun_out/zc3/bench.err || { tail gpurun_out/zc3/bench.err; exit 3; }
python -c "import json; b=json.load(open('gpurun_out/zc3/bench.json')); print(json.dumps(b['host_inclusive'], indent=1))"
