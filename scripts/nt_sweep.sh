set -e
for v in lib lib_nt2 lib_nt16 lib_nt3 lib lib_nt2 lib_nt16 lib_nt3; do
  CUSZ_AMD_LIB=cusz_amd/$v/libcusz_amd.so timeout -k 10 120 python bench.py --config 2 --steps 30 --no-cpu-baseline --no-e2e > gpurun_out/nt_$v.log 2>&1
  python -c "import json,sys;d=json.loads(open('gpurun_out/nt_$v.log').read().strip().splitlines()[-1]);print('$v',d['value'],d['stages_ms'])" | tee -a gpurun_out/nt_summary.txt
done
