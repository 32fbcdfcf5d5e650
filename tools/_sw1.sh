#!/bin/bash
set -u
O=gpurun_out/swT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k shade_threshold -x -q --timeout 200 --timeout-method thread > $O.pytest.log 2>&1 || { mkdir -p gpurun_out; tail -20 $O.pytest.log; exit 1; }
tail -1 $O.pytest.log
bash tools/_sweepT.sh $O/c3.txt "--config 3 --steps 3 --warmup 1" -1 8 12 0x11008 0x11808 0x12008 0x1180c 0x11806 || exit 1
bash tools/_sweepT.sh $O/c4.txt "--config 4 --steps 2 --warmup 1" -1 16 24 32 0x11008 0x12008 || exit 1
bash tools/_sweepT.sh $O/c5.txt "--config 5 --spp 128 --steps 1 --warmup 1" -1 24 32 0x12008 0x11008 || exit 1
cat $O/c3.txt $O/c4.txt $O/c5.txt
