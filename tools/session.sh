#!/bin/bash
# One GPU-box session of named steps; every GPU step has its own time limit and the
# session stops at the first fault, abort or time limit (pytest rc 1 = failed tests
# is reported and the session goes on).
# usage: tools/session.sh <tag> <step...>
#   tests [pytest args]   the GPU suite (or the named test files: tests:file1,file2)
#   ab<C>[f]:<v1>,<v2>,.. A/B of variants/<v>/lib02562rt.so on config C (2, 3, 4; 5 at 128 spp;
#                         f: the fast margin)
#   m<C>[fast] / m4sil    bench line + kernel-trace stats + PMC passes (tools/measure.sh)
#   bench:a,b,..          one bench line (bench.py --no-cpu-baseline a b ..), no profiling
#   n2 / n4 / n8          the same for rank 0's share of an N-rank split (bench.py --rank-share N)
#   wf<C>[f] / wfpmc<C>   the wavefront split's price (tools/wavefront_price.py) / its PMC passes
#   stress                tools/cull_stress.py: configs 3-5 whole frames, every culling mode
#   meshes                tools/mesh_frame.py: the config-3 frame on teapot.obj next to the stand-in
#   sweep<C>[f|s]:T1,..   shading-threshold sweep (tools/sweep_threshold.sh; f fast, s silhouette)
#   scale<C>              tools/scale_probe.py: each rank's share of the N-rank split, N = 1, 2, 4, 8
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
      # ab<C>[f|s]:v1,v2,...  (f: the fast margin, --bsp-cull 2; s: the silhouette bound, --bsp-cull 3)
      c=${step:2:1}; vs=$(echo ${step#*:} | tr , ' '); f=""; fo=""
      [ "${step:3:1}" = "f" ] && { f=f; fo="--bsp-cull 2"; }
      [ "${step:3:1}" = "s" ] && { f=s; fo="--bsp-cull 3"; }
      case $c in 3) o="";; 4) o="--config 4";; 5) o="--config 5 --spp 128";; 2) o="--config 2";; esac
      bash tools/ab.sh $OUT/ab_c$c$f.txt "$o $fo ${AB_OPTS:-}" $vs || { tail -5 $OUT/ab_c$c$f.txt; exit 1; }
      cat $OUT/ab_c$c$f.txt ;;
    wf3|wf5|wf3f|wf5f)
      # the wavefront split's price on the captured ray stream (tools/wavefront_price.py)
      c=${step:2:1}; fo=""; [ "${step:3:1}" = "f" ] && fo="--bsp-cull 2"
      timeout -k 10 600 python tools/wavefront_price.py --config $c $fo > $OUT/wf_c$c${step:3:1}.json 2> $OUT/wf_c$c${step:3:1}.err \
        || { echo "wavefront_price rc=$?"; tail -20 $OUT/wf_c$c${step:3:1}.err; exit 1; }
      cat $OUT/wf_c$c${step:3:1}.json ;;
    wfpmc3|wfpmc5)
      c=${step:5:1}
      PMC_PROG="tools/wavefront_price.py --reps 1" bash tools/profile_pmc.sh $TAG/wf_c$c --config $c || exit 1 ;;
    sweep*)
      # sweep<C>[f]:T1,T2,...  shading thresholds (tools/sweep_threshold.sh; -1 = the default)
      c=${step:5:1}; ts=$(echo ${step#*:} | tr , ' '); f=""; fo=""
      [ "${step:6:1}" = "f" ] && { f=f; fo="--bsp-cull 2"; }
      [ "${step:6:1}" = "s" ] && { f=s; fo="--bsp-cull 3"; }
      case $c in 3) o="";; 4) o="--config 4";; 5) o="--config 5 --spp 128";; 2) o="--config 2";; esac
      bash tools/sweep_threshold.sh $OUT/sweep_c$c$f.txt "$o $fo" $ts || { tail -5 $OUT/sweep_c$c$f.txt; exit 1; }
      cat $OUT/sweep_c$c$f.txt ;;
    scale3|scale4|scale5)
      # per-rank shares of the N-rank tile split, timed one at a time (tools/scale_probe.py)
      c=${step:5:1}; w=""; [ $c = 5 ] && w="--warm 0"
      timeout -k 10 600 python tools/scale_probe.py --config $c $w > $OUT/scale_c$c.txt 2>&1 || { echo "scale_probe rc=$?"; tail -5 $OUT/scale_c$c.txt; exit 1; }
      tail -6 $OUT/scale_c$c.txt ;;
    stress)
      # whole frames of configs 3/4/5 at their BASELINE spp in every culling mode (tools/cull_stress.py)
      timeout -k 10 900 python -u tools/cull_stress.py > $OUT/cull_stress.txt 2>&1 || { echo "cull_stress rc=$?"; tail -20 $OUT/cull_stress.txt; exit 1; }
      grep -E "differ" $OUT/cull_stress.txt ;;
    m3) bash tools/measure.sh $TAG/c3 || exit 1 ;;
    m3fast) bash tools/measure.sh $TAG/c3fast --bsp-cull 2 || exit 1 ;;
    m4) bash tools/measure.sh $TAG/c4 --config 4 --no-cpu-baseline || exit 1 ;;
    m4fast) bash tools/measure.sh $TAG/c4fast --config 4 --no-cpu-baseline --bsp-cull 2 || exit 1 ;;
    m5) bash tools/measure.sh $TAG/c5 --config 5 --no-cpu-baseline || exit 1 ;;
    m5fast) bash tools/measure.sh $TAG/c5fast --config 5 --no-cpu-baseline --bsp-cull 2 || exit 1 ;;
    m2) bash tools/measure.sh $TAG/c2 --config 2 --no-cpu-baseline || exit 1 ;;
    m4sil) bash tools/measure.sh $TAG/c4sil --config 4 --no-cpu-baseline --bsp-cull 3 || exit 1 ;;
    n2|n4|n8) bash tools/measure.sh $TAG/c3$step --no-cpu-baseline --rank-share ${step#n} || exit 1 ;;
    m4auto) bash tools/measure.sh $TAG/c4auto --config 4 --no-cpu-baseline --bsp-cull 4 || exit 1 ;;
    m3bvh) bash tools/measure.sh $TAG/c3bvh --trav BVH --no-cpu-baseline || exit 1 ;;
    m4bvh) bash tools/measure.sh $TAG/c4bvh --config 4 --trav BVH --no-cpu-baseline || exit 1 ;;
    m5bvh) bash tools/measure.sh $TAG/c5bvh --config 5 --trav BVH --no-cpu-baseline ${M5BVH_OPTS:-} || exit 1 ;;
    meshes)
      # the headline frame's shape on the reference's teapot.obj next to the stand-in (tools/mesh_frame.py)
      timeout -k 10 900 python tools/mesh_frame.py --bvh > $OUT/mesh_frame.json 2> $OUT/mesh_frame.err || { echo "mesh_frame rc=$?"; tail -20 $OUT/mesh_frame.err; exit 1; }
      cat $OUT/mesh_frame.json ;;
    bench:*)
      # one bench line, no profiling: bench:--config,4,--bsp-cull,4
      a=$(echo ${step#bench:} | tr , ' ')
      echo "== bench $a" >> $OUT/bench_lines.txt
      timeout -k 10 600 python bench.py --no-cpu-baseline $a > $OUT/bench.tmp 2>&1 || { echo "bench rc=$?"; tail -20 $OUT/bench.tmp; exit 1; }
      grep '^{' $OUT/bench.tmp >> $OUT/bench_lines.txt
      grep '^{' $OUT/bench.tmp | python tools/bench_brief.py ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo session done
