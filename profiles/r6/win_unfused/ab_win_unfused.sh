#!/bin/bash
# A/B of the 16-B hash + window order: fused k_fixed16_win (default) against
# k_fixed16 writing window bytes + k_wo_rank_bytes (SHF_HB_WIN_UNFUSED=1),
# alternating, then one kernel trace of each. Output under gpurun_out/ab_win/.
set -e
mkdir -p gpurun_out/ab_win
for r in 1 2 3; do
  for u in 0 1; do
    SHF_HB_WIN_UNFUSED=$u timeout -k 10 120 python -u bench.py --only hashwin16 --no-cpu --traffic off \
      --no-host-inclusive --steps 50 --warmup 10 > gpurun_out/ab_win/b_${u}_${r}.json 2> gpurun_out/ab_win/b_${u}_${r}.err
  done
done
cd /tmp && export TMPDIR=/tmp
for u in 0 1; do
  SHF_HB_WIN_UNFUSED=$u timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/ab_win/prof_$u \
    -o run -- python3 $GRAFT_REPO_ROOT/bench.py --only hashwin16 --no-cpu --traffic off --no-host-inclusive \
    --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/ab_win/prof_$u.log 2>&1
done
