#!/bin/bash
set -u
O=gpurun_out/swT3; mkdir -p $O
bash tools/_sweepT.sh $O/c3.txt "--config 3 --steps 3 --warmup 1" -1 16 0x12010 || exit 1
bash tools/_sweepT.sh $O/c4.txt "--config 4 --steps 2 --warmup 1" -1 16 || exit 1
bash tools/_sweepT.sh $O/c5.txt "--config 5 --spp 128 --steps 1 --warmup 1" -1 0x12008 || exit 1
bash tools/_sweepT.sh $O/c3f.txt "--config 3 --steps 3 --warmup 1 --bsp-cull 2" -1 || exit 1
cat $O/*.txt
