#!/bin/bash
# Historical: SHFHB_ASM_MIX=1 is now the default, so `asm` equals `base`
# (profiles/r1/ab_asm/ has the A/B from when it was not).
# Mix arithmetic variant (SHFHB_ASM_MIX=1: alignbit rotates, shift-add *5) against
# the compiler's lowering, on every hashing kernel that the bench lines use.
#   python tools/ab.py --prebuild build/ab --variant asm=-DSHFHB_ASM_MIX=1
#   tools/gpu_asm_ab.sh OUTDIR
# A run that fails an ordinary Python check (exit 1, e.g. variants differ) is
# recorded and the next one starts; anything else (fault, abort, time limit) ends
# the script.
set -u
out=$1; mkdir -p $out
V="--variant base= --variant asm=@build/ab/lib_asm.so"
run() {
  local f=$1; shift
  timeout -k 10 200 python tools/ab.py "$@" $V > $out/$f 2>&1
  local rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc=$rc in $f"; exit $rc; fi
  return 0
}
run fixed16.txt --workload fixed16 --n 100000000 --kernel 1 --rounds 7 --reps 5
run fixed256.txt --workload fixed256 --n 25000000 --kernel 2 --rounds 7 --reps 5
run var_span.txt --workload var --n 25000000 --kernel 4 --rounds 7 --reps 5
run var_round.txt --workload var --n 25000000 --kernel 5 --rounds 5 --reps 5
run fixed100_span.txt --workload fixedL --key-len 100 --n 25000000 --kernel 4 --rounds 5 --reps 5
run probe16.txt --workload probe16 --n 10000000 --kernel 0 --rounds 5 --reps 10
echo ok
