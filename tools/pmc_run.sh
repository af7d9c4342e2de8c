#!/bin/bash
# PMC passes over the hashing kernels (run on the GPU box):
#   tools/pmc_run.sh OUTDIR [bench args...]
# Each counter group is its own rocprofv3 pass (--kernel-trace/--stats not mixed with --pmc).
set -u
out=$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_LDS GRBM_COUNT" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum"; do
  i=$((i+1))
  timeout -k 10 400 rocprofv3 --pmc $grp --output-format csv -d "$out/p$i" -o pmc -- python3 bench.py "$@" > "$out/p$i.log" 2>&1 || { echo "pass $i failed rc=$?"; tail -5 "$out/p$i.log"; exit 1; }
done
echo pmc ok
