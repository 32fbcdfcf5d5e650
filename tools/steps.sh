#!/bin/bash
# Named GPU-box steps for one gpurun call, each under its own time limit; the
# call stops at the first failing step (no retries).
# usage: tools/steps.sh <tag> <step> [<step> ...]
#   dist                 tests/test_gpu_bench_dist.py
#   gputests            the whole -m gpu suite
#   pytest:<name>:<paths>  selected GPU tests
#   bench:<name>:<args>  one bench line (args with ',' for spaces) -> <tag>/<name>.json
#   measure:<name>:<args>  tools/measure.sh (bench line, kernel trace, PMC passes)
#   scale:<name>:<args>  tools/scale_probe.py
set -u
TAG=$1; shift
export TMPDIR=/tmp
OUT=gpurun_out/$TAG; mkdir -p $OUT
for step in "$@"; do
  kind=${step%%:*}; rest=${step#*:}; name=${rest%%:*}; args=${rest#*:}; args=${args//,/ }
  [ "$rest" = "$step" ] && { name=$kind; args=""; }
  echo "== $step $(date +%T)"
  case $kind in
    dist)
      timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_dist.py -x -v --timeout 300 --timeout-method thread > $OUT/dist.log 2>&1
      rc=$?; tail -8 $OUT/dist.log; [ $rc -eq 0 ] || exit $rc ;;
    pytest)   # pytest:<name>:<test paths>
      timeout -k 10 900 python -u -m pytest $args -x -v --timeout 300 --timeout-method thread > $OUT/$name.log 2>&1
      rc=$?; tail -4 $OUT/$name.log; grep -E "FAILED|ERROR" $OUT/$name.log | head -20; [ $rc -eq 0 ] || exit $rc ;;
    gputests)
      timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
      rc=$?; tail -3 $OUT/pytest_gpu.log; grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -20; [ $rc -eq 0 ] || exit $rc ;;
    bench)
      timeout -k 10 600 python bench.py $args > $OUT/$name.json 2> $OUT/$name.err || { echo "rc=$?"; tail -20 $OUT/$name.err; exit 1; }
      python tools/bench_brief.py < $OUT/$name.json ;;
    measure)
      bash tools/measure.sh $TAG/$name $args || exit 1 ;;
    scale)
      timeout -k 10 900 python -u tools/scale_probe.py $args > $OUT/$name.txt 2>&1 || { echo "rc=$?"; tail -20 $OUT/$name.txt; exit 1; }
      cat $OUT/$name.txt ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo steps done
