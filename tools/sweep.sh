#!/bin/bash
# parameter sweep of the bench kernel (short runs); usage: tools/sweep.sh <out> <spp> "<opt sets>"
OUT=$1; SPP=$2; shift 2
for o in "$@"; do
  echo "== $o" >> $OUT
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 --warmup 1 --spp $SPP $o 2>&1 | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); t=d['traversal_per_launch']; print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], 'util', d['simd_lane_util'], 'leaf_iters/trip', round(t['leaf_iters']/max(1,t['trips']),3))" >> $OUT || { echo FAIL >> $OUT; exit 1; }
done
