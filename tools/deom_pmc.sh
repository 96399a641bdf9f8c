# DEOM stage kernels: event timing (tools/deom_bench.py) for the XCD block classes, then separate PMC passes
# (FETCH_SIZE; TCC_HIT/TCC_MISS) at 64 hierarchies.  Output under gpurun_out/deom_pmc.
set -e
R=$PWD
OUT=$R/gpurun_out/deom_pmc
mkdir -p $OUT
for x in 0 8; do
  QD_DEOM_XCD=$x timeout -k 10 120 python tools/deom_bench.py 1 16 64 256 >> $OUT/events.jsonl
done
QD_DEOM_ADO_MAJOR=0 QD_DEOM_XCD=8 timeout -k 10 120 python tools/deom_bench.py 64 256 >> $OUT/events.jsonl
cd /tmp && export TMPDIR=/tmp
for x in 0 8; do
  QD_DEOM_XCD=$x DEOM_STEPS=3 timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch_$x -o run -- python3 $R/tools/deom_bench.py 1 64 > $OUT/fetch_$x.log 2>&1
  QD_DEOM_XCD=$x DEOM_STEPS=3 timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/hit_$x -o run -- python3 $R/tools/deom_bench.py 1 64 > $OUT/hit_$x.log 2>&1
done
