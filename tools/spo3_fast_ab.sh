# SPO3 64^3 x 2: latency-shaped mid / x passes (default) vs the generic LDS-staged kernels (QD_SPO3_FAST=0)
set -e
for rep in 1 2; do
  for f in 1 0; do
    QD_SPO3_FAST=$f SPO3_SIZES=32,64,128 timeout -k 10 120 python tools/spo3_bench.py | sed "s/^/fast=$f /"
  done
done
