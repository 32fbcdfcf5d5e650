#!/bin/bash
# Round-4 final measurement sessions.  usage: tools/r4_final.sh <tag> <step...>
#   tests: the GPU suite; c3 / c3fast / c4 / c4fast / c5 / c5fast: bench line,
#   kernel-trace stats and PMC passes (tools/measure.sh) in the certified (default)
#   or fast culling mode; n2 / n4 / n8: rank 0's share of an N-rank split (PMC);
#   scale3/4/5: tools/scale_probe.py
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
    c2) bash tools/measure.sh $TAG/c2 --config 2 --no-cpu-baseline || exit 1 ;;
    c3) bash tools/measure.sh $TAG/c3 || exit 1 ;;
    c3fast) bash tools/measure.sh $TAG/c3fast --bsp-cull 2 || exit 1 ;;
    c4) bash tools/measure.sh $TAG/c4 --config 4 --no-cpu-baseline || exit 1 ;;
    c4fast) bash tools/measure.sh $TAG/c4fast --config 4 --no-cpu-baseline --bsp-cull 2 || exit 1 ;;
    c5) bash tools/measure.sh $TAG/c5 --config 5 --no-cpu-baseline || exit 1 ;;
    c5fast) bash tools/measure.sh $TAG/c5fast --config 5 --no-cpu-baseline --bsp-cull 2 || exit 1 ;;
    n2|n4|n8) SKIP_KS=1 bash tools/measure.sh $TAG/c3$step --no-cpu-baseline --rank-share ${step#n} || exit 1 ;;
    scale3) timeout -k 10 400 python tools/scale_probe.py --config 3 > $OUT/scale_c3.txt 2>&1 || { tail -5 $OUT/scale_c3.txt; exit 1; }; tail -6 $OUT/scale_c3.txt ;;
    scale4) timeout -k 10 400 python tools/scale_probe.py --config 4 > $OUT/scale_c4.txt 2>&1 || { tail -5 $OUT/scale_c4.txt; exit 1; }; tail -6 $OUT/scale_c4.txt ;;
    scale5) timeout -k 10 600 python tools/scale_probe.py --config 5 --warm 0 > $OUT/scale_c5.txt 2>&1 || { tail -5 $OUT/scale_c5.txt; exit 1; }; tail -6 $OUT/scale_c5.txt ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo session done
