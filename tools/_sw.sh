set -u
export TMPDIR=/tmp
OUT=gpurun_out/r01_v11
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py --trav BVH --no-cpu-baseline > $OUT/bench_bvh.json 2> $OUT/bench_bvh.err || { echo "bench rc=$?"; tail -20 $OUT/bench_bvh.err; exit 1; }
python tools/bench_brief.py < $OUT/bench_bvh.json
timeout -k 10 300 python bench.py --config 4 --trav BVH --no-cpu-baseline --steps 1 > $OUT/c4_bvh.json 2> $OUT/c4.err || { echo "c4 rc=$?"; tail -20 $OUT/c4.err; exit 1; }
python tools/bench_brief.py < $OUT/c4_bvh.json
timeout -k 10 400 python bench.py --config 5 --trav BVH --spp 64 --no-cpu-baseline --steps 1 > $OUT/c5_bvh.json 2> $OUT/c5.err || { echo "c5 rc=$?"; tail -20 $OUT/c5.err; exit 1; }
python tools/bench_brief.py < $OUT/c5_bvh.json
echo done
