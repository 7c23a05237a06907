timeout -k 10 600 python bench.py > gpurun_out/bench_full.log 2>&1 || exit $?
tail -1 gpurun_out/bench_full.log
