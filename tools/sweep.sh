#!/bin/bash
# Parameter sweep of the bench kernel (short runs).
# usage: tools/sweep.sh <out> <spp> "<bench opts 1>" "<bench opts 2>" ...
OUT=$1; SPP=$2; shift 2
mkdir -p "$(dirname "$OUT")"
for o in "$@"; do
  echo "== $o" >> $OUT
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 --warmup 1 --spp $SPP $o > $OUT.tmp 2>&1 || { cat $OUT.tmp >> $OUT; echo FAIL >> $OUT; exit 1; }
  grep '^{' $OUT.tmp | python tools/bench_brief.py >> $OUT || { cat $OUT.tmp >> $OUT; exit 1; }
done
rm -f $OUT.tmp
