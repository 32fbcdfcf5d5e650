#!/bin/bash
# Round-4 final measurement sessions.  usage: tools/r4_final.sh <tag> <step...>
#   tests: the GPU suite; c3 / c3fast / c4 / c4fast / c5 / c5fast: bench line,
#   kernel-trace stats and PMC passes (tools/measure.sh) in the certified (default)
#   or fast culling mode
set -u
TAG=$1; shift
export TMPDIR=/tmp
OUT=gpurun_out/$TAG; mkdir -p $OUT
for step in "$@"; do
  case $step in
    tests)
      timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
      rc=$?; tail -3 $OUT/pytest_gpu.log; grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -20
      if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi ;;
    c3) bash tools/measure.sh $TAG/c3 || exit 1 ;;
    c3fast) bash tools/measure.sh $TAG/c3fast --bsp-cull 2 || exit 1 ;;
    c4) bash tools/measure.sh $TAG/c4 --config 4 --no-cpu-baseline || exit 1 ;;
    c4fast) bash tools/measure.sh $TAG/c4fast --config 4 --no-cpu-baseline --bsp-cull 2 || exit 1 ;;
    c5) bash tools/measure.sh $TAG/c5 --config 5 --no-cpu-baseline || exit 1 ;;
    c5fast) bash tools/measure.sh $TAG/c5fast --config 5 --no-cpu-baseline --bsp-cull 2 || exit 1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo session done
