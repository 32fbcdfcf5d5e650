#!/bin/bash
# Same-box comparison of the round-3 tree (abr03/, built from 5037b61) with this
# tree on config 3: usage tools/ab_r03.sh <tag>
# (recreate abr03/: git worktree add /tmp/r03 5037b61, make -C /tmp/r03/02562_raytracer_amd,
#  then copy its 02562_raytracer_amd/, bench.py, oracle/ and tools/ into abr03/; git-ignored)
set -u
export TMPDIR=/tmp
O=$PWD/gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_cull.py tests/test_gpu_cull_grazing.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  (cd abr03 && timeout -k 10 300 python bench.py --config 3 --no-cpu-baseline --steps 3 --warmup 1 > $O/r03_$rep.json 2>$O/err) || exit 1
  echo "r03  $(grep '^{' $O/r03_$rep.json | python tools/bench_brief.py | cut -c1-200)"
  for m in 2 1; do
    timeout -k 10 300 python bench.py --config 3 --no-cpu-baseline --steps 3 --warmup 1 --bsp-cull $m > $O/r04_m${m}_$rep.json 2>$O/err || exit 1
    echo "r04 m$m $(grep '^{' $O/r04_m${m}_$rep.json | python tools/bench_brief.py | cut -c1-200)"
  done
done
