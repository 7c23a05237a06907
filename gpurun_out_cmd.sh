rm -f gpurun_out/bench_config*.log
for c in 1 2 6 7; do timeout -k 10 300 python bench.py --config $c --steps 100 --warmup 2 --no-cpu --check 300 > gpurun_out/bench_config$c.log 2>&1 || exit $?; done
timeout -k 10 300 python bench.py --config 4 --steps 30 --warmup 2 --no-cpu --check 300 > gpurun_out/bench_config4.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config 5 --bindings 125000 --steps 12 --warmup 2 --no-cpu --check 300 > gpurun_out/bench_config5.log 2>&1 || exit $?
