#!/bin/bash
set -u
export TMPDIR=/tmp
O=gpurun_out/ab3; mkdir -p $O
bash tools/ab.sh $O/c3.txt "--config 3 --steps 3 --warmup 1" base tpc12 tpc16 tpc6 base tpc12 || exit 1
bash tools/ab.sh $O/c4.txt "--config 4 --steps 2 --warmup 1" base tpc12 tpc16 || exit 1
bash tools/ab.sh $O/c5.txt "--config 5 --spp 128 --steps 1 --warmup 1" base tpc12 || exit 1
cut -c1-130 $O/c3.txt $O/c4.txt $O/c5.txt
