#!/bin/bash
# A/B of the generic SPO passes (same box): column-tile width floor (QD_SPO_GEN_MINC) and staged kinetic factors
# (QD_SPO_AUX=2), on non-power-of-two SPO2 / SPO3 grids.
mkdir -p gpurun_out
OUT=gpurun_out/spo_gen_ab.txt
: > $OUT
for cfg in "" "QD_SPO_RADIX8=0" "QD_SPO_AUX=2" "QD_SPO_GEN_MINC=2" "QD_SPO_GEN_MINC=4" "QD_SPO_GEN_MINC=8" "QD_SPO_GEN_MINC=4 QD_SPO_AUX=2"; do
  echo "== $cfg" >> $OUT
  env $cfg timeout -k 10 120 python3 tools/spo_any_bench.py 200,500,1000 2d >> $OUT 2>&1 || exit 1
done
cat $OUT
