#!/bin/bash
# leaf-share rule of the per-wave shading threshold (T_hi once the share reaches NUM/DEN; default 1/2)
set -u
export TMPDIR=/tmp
O=gpurun_out/ab11; mkdir -p $O
bash tools/ab.sh $O/c3.txt "--config 3 --steps 3 --warmup 1" base s35 s23 base s35 s23 || exit 1
bash tools/ab.sh $O/c5.txt "--config 5 --spp 128 --steps 1 --warmup 1" base s35 s23 || exit 1
bash tools/ab.sh $O/c4.txt "--config 4 --steps 2 --warmup 1" base s35 || exit 1
cut -c1-100 $O/c3.txt $O/c5.txt $O/c4.txt
