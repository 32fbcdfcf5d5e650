#!/bin/bash
set -u
export TMPDIR=/tmp
O=gpurun_out/ab4; mkdir -p $O
bash tools/ab.sh $O/c3.txt "--config 3 --steps 3 --warmup 1" base xl4 xl8 base || exit 1
cut -c1-130 $O/c3.txt
