#!/bin/bash
# PMC A/B of two variants: VALU instructions, busy and wave cycles per k_path launch (config 3, 1 timed step)
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6l; mkdir -p $OUT
for v in p0 p8; do
  RT_LIBRARY=02562_raytracer_amd/variants/$v/lib02562rt.so timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $OUT/$v -o pmc --output-format csv -- python bench.py --no-cpu-baseline --bsp-cull 1 --steps 1 --warmup 1 > $OUT/$v.log 2>&1 || exit 1
done
echo done
