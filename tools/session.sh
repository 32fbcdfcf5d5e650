#!/bin/bash
# One GPU-box session of named steps; every GPU step has its own time limit and the
# session stops at the first fault, abort or time limit (pytest rc 1 = failed tests
# is reported and the session goes on).
# usage: tools/session.sh <tag> <step...>
#   tests [pytest args]   the GPU suite (or the named test files: tests:file1,file2)
#   ab<C>:<v1>,<v2>,..    A/B of variants/<v>/lib02562rt.so on config C (3, 4; 5 at 128 spp)
#   m<C>[fast]            bench line + kernel-trace stats + PMC passes (tools/measure.sh)
set -u
TAG=$1; shift
export TMPDIR=/tmp
OUT=gpurun_out/$TAG; mkdir -p $OUT
for step in "$@"; do
  case $step in
    tests|tests:*)
      files=tests; [ "$step" != tests ] && files=$(echo ${step#tests:} | tr , ' ')
      timeout -k 10 1000 python -u -m pytest $files -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
      rc=$?; tail -3 $OUT/pytest_gpu.log; grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -20
      if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi ;;
    ab*)
      c=${step:2:1}; vs=$(echo ${step#*:} | tr , ' ')
      case $c in 3) o="";; 4) o="--config 4";; 5) o="--config 5 --spp 128";; 2) o="--config 2";; esac
      bash tools/ab.sh $OUT/ab_c$c.txt "$o ${AB_OPTS:-}" $vs || { tail -5 $OUT/ab_c$c.txt; exit 1; }
      cat $OUT/ab_c$c.txt ;;
    m3) bash tools/measure.sh $TAG/c3 || exit 1 ;;
    m3fast) bash tools/measure.sh $TAG/c3fast --bsp-cull 2 || exit 1 ;;
    m4) bash tools/measure.sh $TAG/c4 --config 4 --no-cpu-baseline || exit 1 ;;
    m4fast) bash tools/measure.sh $TAG/c4fast --config 4 --no-cpu-baseline --bsp-cull 2 || exit 1 ;;
    m5) bash tools/measure.sh $TAG/c5 --config 5 --no-cpu-baseline || exit 1 ;;
    m5fast) bash tools/measure.sh $TAG/c5fast --config 5 --no-cpu-baseline --bsp-cull 2 || exit 1 ;;
    m2) bash tools/measure.sh $TAG/c2 --config 2 --no-cpu-baseline || exit 1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo session done
