#!/bin/bash
# round-4 window-order iteration: scatter variants (timing; tests on the LDS-lean ones)
export TMPDIR=/tmp
o=gpurun_out/${1:-r4c}; mkdir -p $o
for v in 51 52 6; do
SHF_HB_WO_SCATTER=$v timeout -k 10 300 python -u -m pytest tests/test_win_order.py -m gpu -x -q --timeout 120 --timeout-method thread -k "matches_oracle or skewed or fused_fixed16" > $o/pytest_$v.log 2>&1; echo "tests $v: $(tail -1 $o/pytest_$v.log)"
done
B="timeout -k 10 200 python3 bench.py --only winorder,hashwin16 --no-cpu --no-host-inclusive --traffic off --no-verify"
for v in 1 20 264 2128 2192 25 51 52 6; do
  SHF_HB_WO_SCATTER=$v SHF_HB_F16WIN_BLOCK=1024 $B > $o/b_$v.json 2> $o/b_$v.err; echo "scatter $v $(grep '\[bench\]' $o/b_$v.err | tr '\n' ' ')"
done
for b in 0 1024; do
  for v in 20 52 6; do
    SHF_HB_WO_SCATTER=$v SHF_HB_F16WIN_BLOCK=$b $B > $o/h_${b}_${v}.json 2> $o/h_${b}_${v}.err; echo "block $b scatter $v $(grep '\[bench\]' $o/h_${b}_${v}.err | tr '\n' ' ')"
  done
done
