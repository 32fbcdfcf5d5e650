#!/bin/bash
# Build kernel A/B variants: tools/build_variants.sh name1 "DEFS1" name2 "DEFS2" ...
# -> 02562_raytracer_amd/variants/<name>/lib02562rt.so (tools/ab.sh runs them)
cd "$(dirname "$0")/../02562_raytracer_amd" || exit 1
pids=()
while [ $# -ge 2 ]; do
  n=$1; d=$2; shift 2
  mkdir -p variants/$n
  ( make -s BUILD=build_$n LIB=variants/$n/lib02562rt.so DEFS="$d" variants/$n/lib02562rt.so > variants/$n/build.log 2>&1 || echo "build $n failed" ) &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
ls -la variants/*/lib02562rt.so
