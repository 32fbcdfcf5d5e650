#!/bin/bash
set -u
export TMPDIR=/tmp
O=gpurun_out/ab6; mkdir -p $O
bash tools/ab.sh $O/c3.txt "--config 3 --steps 3 --warmup 1" base nocone base nocone || exit 1
bash tools/ab.sh $O/c4.txt "--config 4 --steps 2 --warmup 1" base nocone || exit 1
bash tools/ab.sh $O/c5.txt "--config 5 --spp 128 --steps 1 --warmup 1" base nocone || exit 1
cut -c1-140 $O/c3.txt $O/c4.txt $O/c5.txt
