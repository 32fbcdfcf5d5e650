#!/bin/bash
set -u
export TMPDIR=/tmp
O=gpurun_out/ab5; mkdir -p $O
for v in base rot3 rot5 base; do
  echo "== $v" >> $O/scale.txt
  RT_LIBRARY=02562_raytracer_amd/variants/$v/lib02562rt.so timeout -k 10 300 python tools/scale_probe.py --config 3 --ns 1,8 > $O/tmp.txt 2>&1 || { tail -5 $O/tmp.txt; exit 1; }
  grep chunk $O/tmp.txt >> $O/scale.txt
done
cat $O/scale.txt
