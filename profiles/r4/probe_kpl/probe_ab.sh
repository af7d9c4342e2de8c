#!/bin/bash
export TMPDIR=/tmp
o=gpurun_out/${1:-probe_ab}; mkdir -p $o
for k in 11 12; do
SHF_HB_PROBE_KPL=$k timeout -k 10 300 python -u -m pytest tests/test_gpu_probe.py -m gpu -x -q --timeout 120 --timeout-method thread > $o/pytest_$k.log 2>&1; echo "tests kpl $k: $(tail -1 $o/pytest_$k.log)"
done
for k in 0 11 12 0 11; do
SHF_HB_PROBE_KPL=$k timeout -k 10 300 python3 bench.py --only probe16,probe16_hbm,ceil_probe_rows,ceil_probe_rows_hbm --no-cpu --no-host-inclusive --traffic off > $o/b_$k.json 2> $o/b_$k.err; echo "kpl $k $(grep '\[bench\]' $o/b_$k.err | tr '\n' ' ')"
done
