set -e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_shard.log 2>&1 || { tail -30 gpurun_out/gpu_shard.log; exit 1; }
tail -3 gpurun_out/gpu_shard.log
for tr in BVH BSP; do
tools/ab.sh gpurun_out/ab_shard3.txt "--steps 3 --warmup 1 --trav $tr" base shard
done
