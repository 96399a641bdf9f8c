#!/bin/bash
# A/B of the 2DES 1/8 shard (8,192 members) GEMM block: QD_ENS_BT=64 (split_plan's choice) vs 128 (generated X
# operand, more split-K slabs) and split counts; bench.bench_2des's timed grids after its warm-up, two rounds.
set -e
for rep in 1 2; do
  for cfg in "QD_ENS_BT=64" "QD_ENS_BT=128" "QD_ENS_BT=128 QD_ENS_S=32" "QD_ENS_BT=64 QD_ENS_S=8"; do
    env $cfg timeout -k 10 120 python3 -c "
import sys, json, torch; sys.path.insert(0, '.')
import bench
r, _, _ = bench.bench_2des(torch.device('cuda', 0), 1, 0, 8192, 40)
print(json.dumps({'cfg': '$cfg', 'ms_per_grid': r['ms_per_grid'], 'frac': r['roofline']['frac']}))" 2>&1 | grep cfg
  done
done
