#!/bin/bash
# One GPU-box measurement of a bench workload: the bench line, the kernel-trace
# stats of the same command, and the PMC passes (tools/profile_pmc.sh, short
# runs).  Every GPU step has its own time limit; the script stops at the first
# failure.  Summaries are made afterwards on the CPU (tools/pmc_summary.py).
# usage: tools/measure.sh <tag> [bench args...]
set -u
TAG=$1; shift
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
# the profiled runs name the culling mode the bench line ran: under the default
# RT_BSP_CULL_AUTO the first render's probe launches (the same kernels on a few
# iterations) would otherwise mix into the per-launch averages
m=$(python -c "
import json,sys
d=json.loads([l for l in open('$OUT/bench.json') if l.startswith('{')][-1])['config'].get('bsp_cull') or ''
print({'auto: certified': '--bsp-cull 1', 'auto: silhouette': '--bsp-cull 3'}.get(d.split(' (')[0], ''))")
set -- "$@" $m
echo "profiled with: $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ks -o ks --output-format csv -- python bench.py --no-cpu-baseline "$@" > $OUT/ks.log 2>&1 || { echo "ks rc=$?"; tail -20 $OUT/ks.log; exit 1; }
find $OUT/ks -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
cat $OUT/kernel_stats.csv
if [ "${SKIP_PMC:-0}" = "0" ]; then
  bash tools/profile_pmc.sh $TAG "$@" --steps 1 --warmup 1 || exit 1
fi
echo done
