#!/bin/bash
# window order + seam tests, then the timing experiments
export TMPDIR=/tmp
o=gpurun_out/${1:-r4l}; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_win_order.py tests/test_c_seam.py -m gpu -x -q --timeout 120 --timeout-method thread > $o/pytest.log 2>&1; tail -3 $o/pytest.log
bash tools/gpu_r4c.sh ${1:-r4l}_c
bash tools/gpu_r4k.sh ${1:-r4l}_k
