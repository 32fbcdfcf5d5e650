#!/bin/bash
# W7E3: fast-margin instantiation and shading-phase priority 2 (new) vs the measured build (old)
set -u
export TMPDIR=/tmp
O=gpurun_out/ab13; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_cull.py tests/test_gpu_configs.py tests/test_gpu_w8.py tests/test_gpu_direct.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/ab.sh $O/c2.txt "--config 2 --steps 5 --warmup 2" old new old new || exit 1
bash tools/ab.sh $O/c2f.txt "--config 2 --steps 5 --warmup 2 --bsp-cull 2" old new || exit 1
bash tools/ab.sh $O/c3.txt "--config 3 --steps 3 --warmup 1" old new || exit 1
cut -c1-100 $O/c2.txt $O/c2f.txt $O/c3.txt
