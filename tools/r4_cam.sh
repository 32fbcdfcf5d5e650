#!/bin/bash
# Camera-bound check: the culling tests (grazing and camera rays vs the oracle,
# full frames of configs 2-5, every shader family) and config 3/4/5 bench lines
# in both culling modes.  usage: tools/r4_cam.sh <tag>
set -u
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_cull.py tests/test_gpu_cull_grazing.py tests/test_gpu_cull_fullframe.py -x -v -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; grep -E "FAILED|differ|rays \(" $O/pytest.log | head -20; [ $rc -eq 0 ] || exit $rc
for cfg in 3 4; do for m in 1 2; do
  timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --steps 3 --warmup 1 --bsp-cull $m > $O/b_c${cfg}_m$m.json 2>$O/b.err || { tail -5 $O/b.err; exit 1; }
  echo "c$cfg m$m $(grep '^{' $O/b_c${cfg}_m$m.json | python tools/bench_brief.py | cut -c1-80)"
done; done
for m in 1 2; do
  timeout -k 10 400 python bench.py --config 5 --no-cpu-baseline --steps 1 --warmup 1 --bsp-cull $m > $O/b_c5_m$m.json 2>$O/b.err || { tail -5 $O/b.err; exit 1; }
  echo "c5 m$m $(grep '^{' $O/b_c5_m$m.json | python tools/bench_brief.py | cut -c1-80)"
done
