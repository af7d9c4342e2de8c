#!/bin/bash
# Staged pageable pipeline with the copy-out / copy-in overlap: host tests, then
# 10M x 16-B pageable calls at three stage sizes (tools/diag_pageable_staged.py).
set -e
o=gpurun_out/$1; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_robustness.py tests/test_win_order.py tests/test_gpu_probe.py -m gpu -x -q --timeout 120 --timeout-method thread > $o/pytest.log 2>&1
tail -1 $o/pytest.log
for mb in 32 16 8; do
  timeout -k 10 200 python -u tools/diag_pageable_staged.py --repeats 10 --env SHF_HB_STAGE_MB=$mb --env SHF_HB_TRACE=1 --trace-file $o/trace_$mb.err > $o/stage_$mb.json
  python3 -c "import json; d=json.load(open('$o/stage_$mb.json'))['summary']; print('stage $mb MiB:', d['median'], d['min'], d['max'])"
done
