timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 100 --warmup 2 --no-cpu --check 300 > gpurun_out/final_q.log 2>&1
