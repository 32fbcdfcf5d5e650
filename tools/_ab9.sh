#!/bin/bash
set -u
export TMPDIR=/tmp
O=gpurun_out/ab9; mkdir -p $O
bash tools/ab.sh $O/c3.txt "--config 3 --steps 3 --warmup 1" base prio2 base prio2 || exit 1
bash tools/ab.sh $O/c4.txt "--config 4 --steps 2 --warmup 1" base prio2 || exit 1
bash tools/ab.sh $O/c2.txt "--config 2 --steps 5 --warmup 2" base prio2 || exit 1
cut -c1-110 $O/c3.txt $O/c4.txt $O/c2.txt
