set -u
mkdir -p gpurun_out/tab2
timeout -k 10 300 python -u -m pytest tests/test_gpu_tab.py -x -v --timeout 120 --timeout-method thread > gpurun_out/tab2/pytest.log 2>&1 || { tail -30 gpurun_out/tab2/pytest.log; exit 1; }
tail -3 gpurun_out/tab2/pytest.log
timeout -k 10 300 python tools/ab.py --workload tab --n 1024 --rounds 5 --reps 5 --variant new= --variant old=@build/ab/lib_old.so --variant tab2=@build/ab/lib_tab2.so > gpurun_out/tab2/ab.txt 2>&1 || { tail -5 gpurun_out/tab2/ab.txt; exit 2; }
grep median gpurun_out/tab2/ab.txt
