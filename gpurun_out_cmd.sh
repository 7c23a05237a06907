for rep in 1 2; do
for v in libkp.so libkp_s256w4.so libkp_s512.so; do
  timeout -k 10 300 python bench.py --lib karmada_amd/$v --steps 150 --warmup 2 --no-cpu --check 200 --e2e-reps 0 --inflight 1 > gpurun_out/v.log 2>&1 || exit $?
  tail -1 gpurun_out/v.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['ms_per_step'], d['stages_ms']['sel_all_kernel'], d['parity_checked'], d['parity_bad'])"
done
done
timeout -k 10 300 python bench.py --steps 200 --warmup 2 --no-cpu --check 200 --e2e-reps 0 > gpurun_out/v.log 2>&1 || exit $?
tail -1 gpurun_out/v.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('inflight4 default', d['ms_per_step'], d['serial_ms_per_step'], d['stages_ms']['sel_all_kernel'])"
