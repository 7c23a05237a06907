rm -f gpurun_out/cfgs.jsonl
for c in 1 2 4 6 7; do
  timeout -k 10 300 python bench.py --config $c --steps 100 --warmup 2 --no-cpu --check 300 --e2e-reps 0 > gpurun_out/cfg_$c.log 2>&1 || exit $?
  tail -1 gpurun_out/cfg_$c.log >> gpurun_out/cfgs.jsonl
done
timeout -k 10 300 python bench.py --config 5 --bindings 125000 --steps 12 --warmup 1 --no-cpu --check 300 --e2e-reps 0 > gpurun_out/cfg_5.log 2>&1 || exit $?
tail -1 gpurun_out/cfg_5.log >> gpurun_out/cfgs.jsonl
python3 -c "
import json
for l in open('gpurun_out/cfgs.jsonl'):
    d=json.loads(l); print(d['config']['workload'][:40], d['ms_per_step'], d['serial_ms_per_step'], d['stages_ms']['select_kernels'], d['parity_checked'], d['parity_bad'])"
KP_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 1 --bindings 20000 --no-cpu --check 200 --e2e-reps 0 > gpurun_out/dist2.log 2>&1 || exit $?
tail -1 gpurun_out/dist2.log | cut -c1-400
