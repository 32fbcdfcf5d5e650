#!/bin/bash
# A/B of kernel build variants with their HBM traffic: per variant, the bench
# digest (tools/ab.sh) and two PMC passes (FETCH_SIZE; WRITE_SIZE) over a short
# run, written under gpurun_out/prof/<tag>/<variant>/.
# usage: tools/ab_traffic.sh <out> <tag> "<bench opts>" name1 name2 ...
mkdir -p "$(dirname "$1")"; OUT=$1; TAG=$2; OPTS=$3; shift 3
export TMPDIR=/tmp
for v in "$@"; do
  bash tools/ab.sh $OUT "$OPTS" $v || exit 1
  D=gpurun_out/prof/$TAG/$v; mkdir -p $D
  for P in FETCH_SIZE "WRITE_SIZE SQ_INSTS_VALU"; do
    RT_LIBRARY=02562_raytracer_amd/variants/$v/lib02562rt.so timeout -s KILL 240 rocprofv3 --pmc $P -d $D/p_${P%% *} -o pmc --output-format csv -- python bench.py --no-cpu-baseline --steps 1 --warmup 1 $OPTS > $D/p_${P%% *}.log 2>&1 || { echo "pmc $v $P failed"; tail -5 $D/p_${P%% *}.log; exit 1; }
  done
done
