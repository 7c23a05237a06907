bash gpu_round.sh tests || exit $?
run() { # label lib config bindings steps
  timeout -k 10 300 python bench.py --lib karmada_amd/$2 --config $3 --bindings $4 --steps $5 --warmup 1 --no-cpu --check 300 --e2e-reps 0 > gpurun_out/x_$1.log 2>&1 || exit $?
  tail -1 gpurun_out/x_$1.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$1', d['ms_per_step'], d['stages_ms'], d['parity_checked'], d['parity_bad'])"
}
run c4 libkp.so 4 100000 10
run c5 libkp.so 5 125000 5
run c3 libkp.so 3 100000 50
run c2 libkp.so 2 100000 20
timeout -k 10 300 python bench.py --lib karmada_amd/libkp_stamps.so --config 4 --steps 2 --warmup 1 --no-cpu --check 0 --e2e-reps 0 > gpurun_out/st4.log 2>&1 || exit $?
grep "kp stamps" gpurun_out/st4.log | tail -1
