#!/bin/bash
# Round profile of one bench config (GPU box): kernel-trace stats + FETCH_SIZE and WRITE_SIZE
# passes (separate runs, as MI355X_MICROARCH.md prescribes), summarised into profiles/ by
# prof_summary.py (tag r<round>_c<config>) and profiles/pmc_config<config>.json for bench.py.
# Usage: scripts/pmc_config.sh <tag> <config> [bench args...]
tag=$1; cfg=$2; shift 2
export TMPDIR=/tmp
d=gpurun_out/pmc_$tag
mkdir -p $d
B="python3 bench.py --config $cfg --steps 5 --warmup 2 --profile-only --no-e2e $@"
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $d/stats -o run --output-format csv -- $B > $d/stats.log 2>&1 || exit 1
# counter passes serialise dispatches, so a launch can block until the previous kernel ends: the
# host could then never open the codebook gate the queued upload kernel polls.  Same kernels,
# host-ordered upload instead (CUSZ_AMD_NO_GATE=1).
export CUSZ_AMD_NO_GATE=1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $d/fetch -o run --output-format csv -- $B > $d/fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $d/write -o run --output-format csv -- $B > $d/write.log 2>&1 || exit 1
for x in stats fetch write; do
  f=$(find $d/$x -name "run_*.csv" | head -1); dd=$(dirname "$f"); [ "$dd" != "$d/$x" ] && cp $dd/run_*.csv $d/$x/
done
python3 scripts/prof_summary.py $tag $d/stats $d/fetch $d/write > $d/summary.txt && cp profiles/${tag}_summary.json profiles/pmc_config$cfg.json && cat $d/summary.txt
mkdir -p gpurun_out/profiles_out && cp profiles/${tag}_* profiles/pmc_config$cfg.json gpurun_out/profiles_out/
# the raw traces stay on the box (gpurun_out is copied back only under 64 MiB)
cp $d/summary.txt gpurun_out/profiles_out/${tag}_summary.txt && rm -rf $d
