#!/bin/bash
# WRITE_SIZE / FETCH_SIZE PMC passes of build variants (02562_raytracer_amd/variants/<name>),
# one rocprofv3 run per counter group, on the default bench workload plus extra args.
# usage: tools/pmc_write_variants.sh <tag> "<bench args>" name1 name2 ...
set -u
TAG=$1; ARGS=$2; shift 2
export TMPDIR=/tmp
for v in "$@"; do
  OUT=gpurun_out/prof/$TAG/$v
  mkdir -p $OUT
  i=0
  for P in "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES"; do
    RT_LIBRARY=02562_raytracer_amd/variants/$v/lib02562rt.so timeout -k 10 240 rocprofv3 --pmc $P -d $OUT/pmc$i -o pmc --output-format csv -- python bench.py --no-cpu-baseline $ARGS --steps 1 --warmup 1 > $OUT/pmc$i.log 2>&1 || { echo "$v pass $i rc=$?"; exit 1; }
    i=$((i+1))
  done
  echo "$v done"
done
