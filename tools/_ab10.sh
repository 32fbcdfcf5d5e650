#!/bin/bash
# k_fold variants: LDS-staged loads (flds), reciprocal division (frec), both (fboth)
set -u
export TMPDIR=/tmp
O=gpurun_out/ab10; mkdir -p $O
RT_LIBRARY=02562_raytracer_amd/variants/fboth/lib02562rt.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_render_state.py tests/test_gpu_configs.py tests/test_gpu_w8.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in base flds frec fboth base fboth; do
  RT_LIBRARY=02562_raytracer_amd/variants/$v/lib02562rt.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ks_$v -o ks --output-format csv -- python bench.py --no-cpu-baseline --steps 3 --warmup 1 > $O/b_$v.json 2> $O/b_$v.err || { tail -5 $O/b_$v.err; exit 1; }
  f=$(find $O/ks_$v -name '*kernel_stats.csv' | head -1)
  echo "$v $(grep '^{' $O/b_$v.json | python tools/bench_brief.py | cut -c1-60) | $(grep -h k_fold $f | cut -d, -f2-4)"
  rm -rf $O/ks_$v
done
