#!/bin/bash
# A/B of the alternating-layout 2D passes (QD_SPO_XPOSE=0: in-place passes with strided kinetic loads), two
# alternating rounds on one box, non-power-of-two SPO2 grids.
mkdir -p gpurun_out
OUT=gpurun_out/spo_xpose_ab.txt
: > $OUT
for rep in 1 2; do
  for cfg in "QD_SPO_XPOSE=1" "QD_SPO_XPOSE=0"; do
    echo "== $cfg (round $rep)" >> $OUT
    env $cfg timeout -k 10 120 python3 tools/spo_any_bench.py 200,300,500,1000 2d >> $OUT 2>&1 || exit 1
    env $cfg timeout -k 10 120 python3 tools/spo_any_bench.py 0 3d >> $OUT 2>&1 || exit 1
  done
done
cat $OUT
