#!/bin/bash
# A/B timing of kernel build variants (02562_raytracer_amd/variants/<name>/lib02562rt.so,
# selected through RT_LIBRARY), each with the default bench workload.
# usage: tools/ab.sh <out> "<bench opts>" name1 name2 ...
mkdir -p "$(dirname "$1")"; OUT=$1; OPTS=$2; shift 2
for v in "$@"; do
  echo "== $v $OPTS" >> $OUT
  RT_LIBRARY=02562_raytracer_amd/variants/$v/lib02562rt.so timeout -k 10 300 python bench.py --no-cpu-baseline $OPTS > $OUT.tmp 2>&1 || { cat $OUT.tmp >> $OUT; echo FAIL >> $OUT; exit 1; }
  grep '^{' $OUT.tmp | python tools/bench_brief.py >> $OUT || { cat $OUT.tmp >> $OUT; exit 1; }
done
rm -f $OUT.tmp
