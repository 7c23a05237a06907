bash gpu_round.sh tests || exit $?
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 150 --warmup 2 --no-cpu --check 2000 --e2e-reps 0 --inflight 1 > gpurun_out/v.log 2>&1 || exit $?
  tail -1 gpurun_out/v.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('serial', d['ms_per_step'], d['stages_ms'], d['parity_checked'], d['parity_bad'])"
done
