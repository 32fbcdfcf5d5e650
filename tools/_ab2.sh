#!/bin/bash
set -u
export TMPDIR=/tmp
O=gpurun_out/ab2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_cull.py tests/test_gpu_cull_grazing.py -x -q -s --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
grep -E "passed|differ" $O/pytest.log
bash tools/ab.sh $O/c3.txt "--config 3 --steps 3 --warmup 1 --bsp-cull 1" pk nopk pk nopk || exit 1
bash tools/ab.sh $O/c3.txt "--config 3 --steps 3 --warmup 1 --bsp-cull 2" fastf pk || exit 1
bash tools/ab.sh $O/c4.txt "--config 4 --steps 2 --warmup 1 --bsp-cull 1" pk nopk || exit 1
cut -c1-150 $O/c3.txt $O/c4.txt
