set -u
export TMPDIR=/tmp
OUT=gpurun_out/r01_v10
mkdir -p $OUT
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 python bench.py --trav BVH > $OUT/bench_bvh.json 2> $OUT/bench_bvh.err || { echo "bench rc=$?"; tail -20 $OUT/bench_bvh.err; exit 1; }
cat $OUT/bench_bvh.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ks -o ks --output-format csv -- python bench.py --no-cpu-baseline --trav BVH > $OUT/ks.log 2>&1 || { echo "ks rc=$?"; tail -20 $OUT/ks.log; exit 1; }
find $OUT/ks -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats_bvh.csv \;
cat $OUT/kernel_stats_bvh.csv
bash tools/profile_pmc.sh r01_v10_bvh --trav BVH || exit 1
echo done
