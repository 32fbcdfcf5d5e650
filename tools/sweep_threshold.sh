#!/bin/bash
# Shading-threshold sweep of one workload: tools/sweep_threshold.sh <out> "<bench opts>" T1 T2 ...
mkdir -p "$(dirname "$1")"; OUT=$1; OPTS=$2; shift 2
for t in "$@"; do
  echo "== T=$t $OPTS" >> $OUT
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 --warmup 1 $OPTS --shade-threshold $t > $OUT.tmp 2>&1 || { cat $OUT.tmp >> $OUT; echo FAIL >> $OUT; exit 1; }
  grep '^{' $OUT.tmp | python tools/bench_brief.py >> $OUT || { cat $OUT.tmp >> $OUT; exit 1; }
done
rm -f $OUT.tmp
