#!/bin/bash
# the fast-margin instantiation of W9E1's BSP k_path: culling tests, then bench lines
set -u
export TMPDIR=/tmp
O=gpurun_out/ab7; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_cull.py tests/test_gpu_cull_grazing.py tests/test_gpu_cull_fullframe.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for a in "--config 3 --steps 3 --warmup 1 --bsp-cull 2" "--config 3 --steps 3 --warmup 1" "--config 4 --steps 2 --warmup 1 --bsp-cull 2" "--config 5 --steps 1 --warmup 1 --bsp-cull 2"; do
  timeout -k 10 400 python bench.py --no-cpu-baseline $a > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
  echo "$a: $(grep '^{' $O/b.json | python tools/bench_brief.py | cut -c1-120)"
done
