#!/bin/bash
# shading-threshold sweep on the certified walk: tools/_sweepT.sh <out> "<bench opts>" T1 T2 ...
set -u
export TMPDIR=/tmp
OUT=$1; OPTS=$2; shift 2; mkdir -p $(dirname $OUT)
for t in "$@"; do
  echo "== T $t $OPTS" >> $OUT
  timeout -k 10 400 python bench.py --no-cpu-baseline $OPTS --shade-threshold $t > $OUT.tmp 2>&1 || { tail -5 $OUT.tmp >> $OUT; echo FAIL >> $OUT; exit 1; }
  grep '^{' $OUT.tmp | python tools/bench_brief.py | cut -c1-150 >> $OUT
done
rm -f $OUT.tmp
