for v in "" "KP_SEL_WIDE=1" "KP_SEL_THREADS=256"; do
  env $v timeout -k 10 300 python bench.py --steps 100 --warmup 2 --no-cpu --check 200 --e2e-reps 0 --inflight 1 > gpurun_out/v.log 2>&1 || exit $?
  tail -1 gpurun_out/v.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['ms_per_step'], d['stages_ms']['sel_all_kernel'], d['parity_checked'], d['parity_bad'])"
done
