#!/bin/bash
# Runtime-knob sweep of one workload: tools/sweep_knobs.sh <out> "<bench opts>" "<knobs 1>" "<knobs 2>" ...
# e.g. tools/sweep_knobs.sh o.txt "--config 5 --spp 16" "--shade-threshold 32" "--shade-threshold 24"
mkdir -p "$(dirname "$1")"; OUT=$1; OPTS=$2; shift 2
for k in "$@"; do
  echo "== $k $OPTS" >> $OUT
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 --warmup 1 $OPTS $k > $OUT.tmp 2>&1 || { cat $OUT.tmp >> $OUT; echo FAIL >> $OUT; exit 1; }
  grep '^{' $OUT.tmp | python tools/bench_brief.py >> $OUT || { cat $OUT.tmp >> $OUT; exit 1; }
done
rm -f $OUT.tmp
