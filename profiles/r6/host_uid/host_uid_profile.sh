#!/bin/bash
# Kernel and copy trace of the host-memory pipeline (10M x 16-B keys, UID parts
# and hashes from pageable buffers; tools/host_uid_sweep.py), so a call's time
# can be split into kernels, copy-engine transfers and the rest.
# Output: gpurun_out/host_uid_prof/ (csv traces), then tools/rocprof_summary.py.
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/host_uid_prof
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $out -o run -- \
  python3 $GRAFT_REPO_ROOT/tools/host_uid_sweep.py --set default: --rounds 1 --reps 5 --modes uid,hash \
  > $out/sweep.json 2> $out/sweep.err
