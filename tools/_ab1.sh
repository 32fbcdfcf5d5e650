#!/bin/bash
set -u
export TMPDIR=/tmp
O=gpurun_out/ab1; mkdir -p $O
bash tools/ab.sh $O/c3.txt "--config 3 --steps 3 --warmup 1 --bsp-cull 2" base fastf || exit 1
bash tools/ab.sh $O/c3.txt "--config 3 --steps 3 --warmup 1 --bsp-cull 1" base nocam || exit 1
(cd abr03 && timeout -k 10 300 python bench.py --config 3 --no-cpu-baseline --steps 3 --warmup 1 > ../$O/r03.json 2>&1) || exit 1
echo "== r03" >> $O/c3.txt; grep '^{' $O/r03.json | python tools/bench_brief.py >> $O/c3.txt
cut -c1-120 $O/c3.txt
