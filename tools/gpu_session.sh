#!/bin/bash
# One GPU-box session: the GPU test suite, then measurement steps.  A test
# failure (pytest rc 1) is reported and the measurements still run; any other
# failure (fault, abort, time limit) ends the session.
# usage: tools/gpu_session.sh <tag> [step ...]   steps: tests | build | c3 | c5 | c4 | c2 | bvh3 | probe
set -u
TAG=$1; shift
export TMPDIR=/tmp
OUT=gpurun_out/$TAG; mkdir -p $OUT
for step in "$@"; do
  case $step in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
      rc=$?; tail -3 $OUT/pytest_gpu.log; grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -20
      if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi ;;
    build)
      timeout -k 10 300 python tools/build_bench.py --out $OUT/build_gpu.jsonl > $OUT/build.log 2>&1 || { echo "build bench rc=$?"; tail -5 $OUT/build.log; exit 1; } ;;
    c3) bash tools/measure.sh $TAG/c3 || exit 1 ;;
    bvh3) SKIP_PMC=${SKIP_PMC:-0} bash tools/measure.sh $TAG/bvh3 --trav BVH || exit 1 ;;
    c2) bash tools/measure.sh $TAG/c2 --config 2 || exit 1 ;;
    c4) bash tools/measure.sh $TAG/c4 --config 4 --spp 64 || exit 1 ;;
    c5) bash tools/measure.sh $TAG/c5 --config 5 --spp 64 --shade-threshold 32 || exit 1 ;;
    probe) timeout -k 10 40 ./tools/probes/issue_probe > $OUT/issue_probe.txt 2>&1; rc=$?; cat $OUT/issue_probe.txt; [ $rc -eq 0 ] || exit $rc ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo session done
