#!/bin/bash
# GPU-box driver for one gpurun call: smoke, GPU parity tests, short bench.
# Stops at the first step that ends in a fault/abort/timeout (exit code >1).
mkdir -p gpurun_out
ROOT=$(pwd)
step() {
  local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
for s in "$@"; do
  case $s in
    smoke) step smoke 300 python -c 'import __graft_entry__ as g; g.smoke()' ;;
    tests) step gpu_tests 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    bench_small) step bench_small 300 python bench.py --steps 3 --warmup 1 --bindings 5000 --no-cpu ;;
    bench) step bench 600 python bench.py ;;
    benchq) step benchq 300 python bench.py --steps 100 --warmup 2 --no-cpu --check 300 ;;
    benchq_notop) KP_TOP=0 step benchq_notop 300 python bench.py --steps 100 --warmup 2 --no-cpu --check 300 --e2e-reps 0 ;;
    cfg_*) c=${s#cfg_}; b=100000; [ "$c" = 5 ] && b=125000
           step bench_cfg$c 300 python bench.py --config $c --bindings $b --steps 20 --warmup 2 --no-cpu --check 300 --e2e-reps 0 ;;
    bench_rows) KP_PAIR_ROWS=1 step bench_rows 300 python bench.py --steps 100 --warmup 2 --no-cpu --check 300 --e2e-reps 0 ;;
    cpubase) step cpubase 900 python tools/cpu_baseline.py --budget 8 ;;
    capsweep) for c in 256 384 768 1024; do KP_TOP_CAP=$c step cap_$c 300 python bench.py --steps 50 --warmup 2 --no-cpu --check 100 --e2e-reps 0; done ;;
    sweep) for t in 256 512; do KP_SEL_THREADS=$t step sweep_$t 300 python bench.py --steps 3 --warmup 1 --no-cpu; done ;;
    chunks) for c in 4096 8192 16384 32768 200000; do KP_CHUNK=$c step chunk_$c 300 python bench.py --steps 5 --warmup 1 --no-cpu; done ;;
    configs) for c in 2 4 6; do step bench_config$c 300 python bench.py --config $c --steps 3 --warmup 1 --no-cpu; done
             step bench_config5 300 python bench.py --config 5 --bindings 125000 --steps 3 --warmup 1 --no-cpu ;;
    stampsc_*) c=${s#stampsc_}; b=100000; [ "$c" = 5 ] && b=125000
           step stamps_cfg$c 300 python bench.py --lib karmada_amd/libkp_stamps.so --config $c --bindings $b --steps 2 --warmup 1 --no-cpu --check 0 --inflight 1 --e2e-reps 0 ;;
    stamps) step stamps 300 python bench.py --lib karmada_amd/libkp_stamps.so --steps 2 --warmup 1 --no-cpu --check 0 ;;
    lib_*) n=${s#lib_}; step bench_$n 300 python bench.py --lib karmada_amd/libkp_$n.so --steps 50 --warmup 2 --no-cpu --check 200 ;;
    libst_*) n=${s#libst_}; step stamps_$n 300 python bench.py --lib karmada_amd/libkp_$n.so --steps 2 --warmup 1 --no-cpu --check 0 ;;
    prof_sq) step prof_sq 600 bash -c "cd /tmp && export TMPDIR=/tmp && rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d $ROOT/gpurun_out/prof_sq -o sq -- python3 $ROOT/bench.py --steps 1 --warmup 0 --no-cpu" ;;
    prof_kt) step prof_kt 600 bash -c "cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/prof_kt -o kt -- python3 $ROOT/bench.py --steps 5 --warmup 1 --no-cpu --inflight 1 --e2e-reps 0" ;;
    prof_fetch) step prof_fetch 600 bash -c "cd /tmp && export TMPDIR=/tmp && rocprofv3 --pmc FETCH_SIZE --output-format csv -d $ROOT/gpurun_out/prof_fetch -o f -- python3 $ROOT/bench.py --steps 2 --warmup 0 --no-cpu" ;;
    prof_write) step prof_write 600 bash -c "cd /tmp && export TMPDIR=/tmp && rocprofv3 --pmc WRITE_SIZE --output-format csv -d $ROOT/gpurun_out/prof_write -o w -- python3 $ROOT/bench.py --steps 2 --warmup 0 --no-cpu" ;;
    dist2) KP_DIST_BACKEND=gloo step dist2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --bindings 20000 ;;
    prof_kt45) for c in 4 5; do step prof_kt$c 600 bash -c "cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/prof_kt$c -o kt -- python3 $ROOT/bench.py --config $c --bindings 100000 --steps 3 --warmup 1 --no-cpu --inflight 1 --e2e-reps 0 --check 0"; done ;;
    pmc_*) c=${s#pmc_}; b=100000; [ "$c" = 5 ] && b=125000
           step pmc_cfg$c 900 bash tools/gpu/prof_pmc.sh cfg$c --config $c --bindings $b ;;
    prof_l2) step prof_l2 600 bash -c "cd /tmp && export TMPDIR=/tmp && rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $ROOT/gpurun_out/prof_l2 -o l -- python3 $ROOT/bench.py --steps 2 --warmup 0 --no-cpu" ;;
  esac
done
