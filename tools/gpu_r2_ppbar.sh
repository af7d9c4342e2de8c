set -e
bash tools/gpu_span_ab2.sh gpurun_out/ab_ppbar "new" "" "8:512 260:260 200:400 64:448 8:256"
timeout -k 10 200 python tools/ab.py --workload tab --n 1024 --rounds 5 --reps 5 --variant base= --variant new=@build/ab/lib_new.so --variant tabsync=@build/ab/lib_tabsync.so > gpurun_out/ab_ppbar/tab.txt 2>&1
grep median gpurun_out/ab_ppbar/tab.txt
