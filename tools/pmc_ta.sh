#!/bin/bash
set -u
export TMPDIR=/tmp
OUT=gpurun_out/prof/ta
mkdir -p $OUT
PASSES=(
  "TA_TA_BUSY_sum TA_BUFFER_TOTAL_CYCLES_sum GRBM_GUI_ACTIVE"
  "TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum"
  "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum"
  "TCP_TCP_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TD_TCP_STALL_CYCLES_sum"
)
i=0
for P in "${PASSES[@]}"; do
  timeout -s KILL 120 rocprofv3 --pmc $P -d $OUT/pmc$i -o pmc --output-format csv -- python bench.py --no-cpu-baseline --spp 64 > $OUT/pmc$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/pmc$i.log; exit $rc; fi
  i=$((i+1))
done
