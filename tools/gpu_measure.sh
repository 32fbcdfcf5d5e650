#!/bin/bash
# One GPU-box measurement pass: parity suite, default bench line, kernel-trace
# stats of the same bench command, PMC passes.  Every GPU step has its own time
# limit; the script stops at the first failure.
# usage: tools/gpu_measure.sh <tag> [--skip-tests] [--skip-pmc]
set -u
TAG=$1; shift
SKIP_TESTS=0; SKIP_PMC=0
for a in "$@"; do
  case $a in --skip-tests) SKIP_TESTS=1;; --skip-pmc) SKIP_PMC=1;; esac
done
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ $SKIP_TESTS -eq 0 ]; then
  timeout -k 10 600 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
fi
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ks -o ks --output-format csv -- python bench.py --no-cpu-baseline > $OUT/ks.log 2>&1 || { echo "ks rc=$?"; tail -20 $OUT/ks.log; exit 1; }
find $OUT/ks -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
cat $OUT/kernel_stats.csv
if [ $SKIP_PMC -eq 0 ]; then
  bash tools/profile_pmc.sh $TAG/pmc || exit 1
fi
echo done
