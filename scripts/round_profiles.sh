#!/bin/bash
# Round-end evidence on the GPU box: bench lines and rocprof summaries per config.
#   scripts/round_profiles.sh <round tag, e.g. r04> <config> [<config> ...]
# -> gpurun_out/profiles_out/{<tag>_bench_config<N>.json, <tag>_c<N>_*}, pmc_config<N>.json
cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift
mkdir -p gpurun_out/profiles_out
for cfg in "$@"; do
  echo "== config $cfg $(date +%T)"
  timeout -k 10 300 python3 bench.py --config "$cfg" > gpurun_out/bench_c$cfg.log 2>&1 || exit 1
  tail -1 gpurun_out/bench_c$cfg.log > gpurun_out/profiles_out/${tag}_bench_config$cfg.json
  scripts/pmc_config.sh ${tag}_c$cfg "$cfg" || exit 1
  rm -rf gpurun_out/pmc_${tag}_c$cfg  # raw rocprof output (the summaries are in profiles_out)
done
