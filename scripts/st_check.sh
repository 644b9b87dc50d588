set -e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_st.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_st.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench_st.log 2>&1
for c in 3 1 5; do
  timeout -k 10 120 python bench.py --config $c --steps 20 --no-cpu-baseline --no-e2e > gpurun_out/stc_$c.log 2>&1
done
