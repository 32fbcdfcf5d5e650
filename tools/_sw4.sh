#!/bin/bash
set -u
O=gpurun_out/swT4; mkdir -p $O
bash tools/_sweepT.sh $O/c2.txt "--config 2 --steps 5 --warmup 2" -1 16 32 40 0x12010 0x11810 -1 || exit 1
cat $O/c2.txt
