set -u
export TMPDIR=/tmp
OUT=gpurun_out/r01v13c
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_bvh_stack.py -x -q --timeout 120 --timeout-method thread > $OUT/stack_2pop.log 2>&1 || { echo "2pop rc=$?"; tail -30 $OUT/stack_2pop.log; exit 1; }
tail -1 $OUT/stack_2pop.log
RT_LIBRARY=02562_raytracer_amd/variants/1pop/lib02562rt.so timeout -k 10 300 python -u -m pytest tests/test_gpu_bvh_stack.py -x -q --timeout 120 --timeout-method thread > $OUT/stack_1pop.log 2>&1 || { echo "1pop rc=$?"; tail -30 $OUT/stack_1pop.log; exit 1; }
tail -1 $OUT/stack_1pop.log
timeout -k 10 300 python bench.py --trav BVH --no-cpu-baseline > $OUT/bench_bvh.json 2> $OUT/bench_bvh.err || { echo "bench rc=$?"; tail -20 $OUT/bench_bvh.err; exit 1; }
cat $OUT/bench_bvh.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ks -o ks --output-format csv -- python bench.py --trav BVH --no-cpu-baseline > $OUT/ks.log 2>&1 || { echo "ks rc=$?"; tail -20 $OUT/ks.log; exit 1; }
find $OUT/ks -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
head -3 $OUT/kernel_stats.csv
