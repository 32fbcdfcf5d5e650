#!/bin/bash
# Round-4 measurement session: configs 3-5 in both culling modes (bench lines),
# and the kernel-trace + PMC passes of the default (certified) config-3 line.
# usage: tools/r4_measure.sh <tag> [c3pmc] [c4] [c5] [c3fast]
set -u
TAG=$1; shift
export TMPDIR=/tmp
OUT=gpurun_out/$TAG; mkdir -p $OUT
for step in "$@"; do
  case $step in
    c3pmc) bash tools/measure.sh $TAG/c3 || exit 1 ;;
    c3fastpmc) bash tools/measure.sh $TAG/c3fast --bsp-cull 2 || exit 1 ;;
    c4) for m in 1 2; do timeout -k 10 400 python bench.py --config 4 --no-cpu-baseline --bsp-cull $m --steps 3 --warmup 1 > $OUT/bench_c4_m$m.json 2> $OUT/bench_c4_m$m.err || { echo "c4 m$m rc=$?"; tail -5 $OUT/bench_c4_m$m.err; exit 1; }; head -c 300 $OUT/bench_c4_m$m.json; echo; done ;;
    c5) for m in 2 1; do timeout -k 10 600 python bench.py --config 5 --no-cpu-baseline --bsp-cull $m --steps 1 --warmup 1 --progress > $OUT/bench_c5_m$m.json 2> $OUT/bench_c5_m$m.err || { echo "c5 m$m rc=$?"; tail -5 $OUT/bench_c5_m$m.err; exit 1; }; head -c 300 $OUT/bench_c5_m$m.json; echo; done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo session done
