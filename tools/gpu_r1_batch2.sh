#!/bin/bash
# Round-1 experiment batch on one GPU box: full-size parity (configs 2/3/4), the
# mix-arithmetic / sorted-span / probe keys-per-lane A/B runs and the host
# pipeline shape sweep. Stops at the first step that faults or times out.
#   tools/gpu_r1_batch2.sh OUTDIR
set -u
o=$1; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 300 --timeout-method thread \
  > $o/fullsize.log 2>&1 || { echo "fullsize failed"; tail -20 $o/fullsize.log; exit 1; }
tools/gpu_asm_ab.sh $o/asm || { echo "asm ab stopped"; exit 2; }
tools/gpu_sort_ab.sh $o/sort || { echo "sort ab stopped"; exit 3; }
timeout -k 10 200 python tools/ab.py --workload probe16 --n 10000000 --kernel 0 --rounds 7 --reps 10 \
  --variant base= --variant head=@build/ab/lib_head.so --variant p2=@build/ab/lib_p2.so --variant p4=@build/ab/lib_p4.so \
  > $o/probe_kpl.txt 2>&1 || { echo "probe ab failed"; exit 4; }
timeout -k 10 300 python tools/host_pipeline_sweep.py > $o/host_pipeline_sweep.txt 2>&1 || { echo "sweep failed"; exit 5; }
echo batch ok
