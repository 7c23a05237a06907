rm -rf gpurun_out/prof_kt4
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_kt4 -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --config 4 --steps 5 --warmup 1 --no-cpu --inflight 1 --e2e-reps 0 --check 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_kt4.log 2>&1
