#!/bin/bash
set -u
export TMPDIR=/tmp
O=gpurun_out/m2; mkdir -p $O
for a in "--config 2" "--config 2 --bsp-cull 2" "--config 2 --bsp-cull 0" "--trav BVH"; do
  timeout -k 10 400 python bench.py --no-cpu-baseline --steps 3 --warmup 1 $a > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
  echo "$a: $(grep '^{' $O/b.json | python tools/bench_brief.py | cut -c1-150)"
done
