set -e
for c in 2 3; do
for v in lib lib_st2 lib_st3 lib lib_st2 lib_st3; do
  CUSZ_AMD_LIB=cusz_amd/$v/libcusz_amd.so timeout -k 10 120 python bench.py --config $c --steps 30 --no-cpu-baseline --no-e2e > gpurun_out/st_$v.log 2>&1
  python -c "import json;d=json.loads(open('gpurun_out/st_$v.log').read().strip().splitlines()[-1]);s=d['stages_ms'];print($c,'$v',d['value'],s['compress'],s['decode'],s['decompress'])" | tee -a gpurun_out/st_summary.txt
done; done
