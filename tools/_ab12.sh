#!/bin/bash
# 12-B sample records with the primary ids written by k_path (rec12) vs 16-B records (rec16)
set -u
export TMPDIR=/tmp
O=gpurun_out/ab12; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_render_state.py tests/test_gpu_configs.py tests/test_gpu_async_fold.py tests/test_gpu_w8.py tests/test_gpu_cull.py tests/test_gpu_bench_dist.py tests/test_gpu_comm.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in rec16 rec12 rec16 rec12 rec16 rec12; do
  RT_LIBRARY=02562_raytracer_amd/variants/$v/lib02562rt.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ks_$v -o ks --output-format csv -- python bench.py --no-cpu-baseline --steps 3 --warmup 1 > $O/b_$v.json 2> $O/b_$v.err || { tail -5 $O/b_$v.err; exit 1; }
  f=$(find $O/ks_$v -name '*kernel_stats.csv' | head -1)
  echo "$v $(grep '^{' $O/b_$v.json | python tools/bench_brief.py | cut -c1-60) | fold $(grep -h k_fold $f | cut -d, -f4) | path $(grep -h 'k_path<4, 0, false, true>' $f | cut -d, -f4)"
  rm -rf $O/ks_$v
done
bash tools/ab.sh $O/c4.txt "--config 4 --steps 2 --warmup 1" rec16 rec12 || exit 1
bash tools/ab.sh $O/c2.txt "--config 2 --steps 5 --warmup 2" rec16 rec12 || exit 1
cut -c1-90 $O/c4.txt $O/c2.txt
