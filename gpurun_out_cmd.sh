timeout -k 10 300 python bench.py --config 4 --lib karmada_amd/libkp_stamps.so --steps 2 --warmup 1 --no-cpu --check 0 --inflight 1 --e2e-reps 0 > gpurun_out/st4.log 2>&1 || exit $?
