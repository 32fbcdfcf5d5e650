#!/bin/bash
set -u
O=gpurun_out/swT2; mkdir -p $O
bash tools/_sweepT.sh $O/c3.txt "--config 3 --steps 3 --warmup 1" 12 0x1200c 16 -1 || exit 1
bash tools/_sweepT.sh $O/c4.txt "--config 4 --steps 2 --warmup 1" 0x1200c 12 20 || exit 1
bash tools/_sweepT.sh $O/c5.txt "--config 5 --spp 128 --steps 1 --warmup 1" 0x1200c || exit 1
bash tools/_sweepT.sh $O/c3f.txt "--config 3 --steps 3 --warmup 1 --bsp-cull 2" -1 0x1200c || exit 1
bash tools/_sweepT.sh $O/c4f.txt "--config 4 --steps 2 --warmup 1 --bsp-cull 2" -1 0x1200c || exit 1
bash tools/_sweepT.sh $O/c5f.txt "--config 5 --spp 128 --steps 1 --warmup 1 --bsp-cull 2" -1 0x1200c || exit 1
cat $O/*.txt
