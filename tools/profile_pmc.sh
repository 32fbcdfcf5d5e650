#!/bin/bash
# PMC passes over a short bench run (one counter group per rocprofv3 run, as
# MI355X_MICROARCH.md "rocprofv3 PMC slots" requires).  Writes gpurun_out/prof/<tag>/pmc<i>/.
# usage: tools/profile_pmc.sh <tag> [bench args...]
# (PMC_PROG: the python program and its fixed arguments, default "bench.py --no-cpu-baseline")
set -u
TAG=$1; shift
export TMPDIR=/tmp
OUT=gpurun_out/prof/$TAG
mkdir -p $OUT
PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
  "SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR"
  "FETCH_SIZE"
  "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
  "GRBM_GUI_ACTIVE TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum SQ_LDS_BANK_CONFLICT"
)
i=0
for P in "${PASSES[@]}"; do
  timeout -k 10 240 rocprofv3 --pmc $P -d $OUT/pmc$i -o pmc --output-format csv -- python ${PMC_PROG:-bench.py --no-cpu-baseline} "$@" > $OUT/pmc$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
  i=$((i+1))
done
