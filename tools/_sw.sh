set -u
export TMPDIR=/tmp
OUT=gpurun_out/r01v14
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_bvh_stack.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "bvh or BVH" > $OUT/bvh_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/bvh_tests.log; exit 1; }
tail -1 $OUT/bvh_tests.log
bash tools/ab.sh $OUT/ab.txt "--trav BVH" 2pop bf 2pop bf || exit 1
cat $OUT/ab.txt | cut -c1-80
