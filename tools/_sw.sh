set -u
export TMPDIR=/tmp
OUT=gpurun_out/r01v18b
mkdir -p $OUT
( while sleep 20; do date >> $OUT/heartbeat.txt; done ) &
HB=$!
trap "kill $HB" EXIT
for a in "5 BVH" "4 BSP" "2 BSP"; do
  set -- $a
  timeout -k 10 500 python -u bench.py --config $1 --trav $2 --no-cpu-baseline > $OUT/c$1_$2.json 2> $OUT/c$1_$2.err || { echo "config $1 $2 rc=$?"; tail -20 $OUT/c$1_$2.err; exit 1; }
  python tools/bench_brief.py < $OUT/c$1_$2.json | cut -c1-100
done
