#!/bin/bash
# cooperative LDS-staged k_fold (RT_FOLD_LDS=1) against the default
set -u
export TMPDIR=/tmp
O=gpurun_out/ab8; mkdir -p $O
for v in base flds; do
  RT_LIBRARY=02562_raytracer_amd/variants/$v/lib02562rt.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ks_$v -o ks --output-format csv -- python bench.py --no-cpu-baseline --steps 3 --warmup 1 > $O/b_$v.json 2> $O/b_$v.err || { tail -5 $O/b_$v.err; exit 1; }
  echo "$v $(grep '^{' $O/b_$v.json | python tools/bench_brief.py | cut -c1-80)"
  for f in $(find $O/ks_$v -name '*kernel_stats.csv'); do grep -h "k_fold" $f | cut -c1-100; done
done
