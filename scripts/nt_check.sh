set -e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_nt.log 2>&1
for c in 2 3 1; do
  timeout -k 10 120 python bench.py --config $c --steps 30 --no-cpu-baseline --no-e2e > gpurun_out/ntc_$c.log 2>&1
  python -c "import json;d=json.loads(open('gpurun_out/ntc_$c.log').read().strip().splitlines()[-1]);print($c,d['value'],d['ms_per_step'],d['stages_ms'])" | tee -a gpurun_out/ntc_summary.txt
done
