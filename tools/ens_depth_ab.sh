# 2DES 1/8 shard (64-blocks) with the operand loads one K-tile ahead (QD_ENS_DEPTH=1) vs two (=2): bench 2DES leg.
set -e
for rep in 1 2; do
  for x in 2 1; do
    QD_ENS_DEPTH=$x timeout -k 10 150 python bench.py --steps 2 --warmup 1 --batch 4 --no-cpu --t2 0 --no-redfield \
      --no-superop --no-spo --no-spo3 --no-deom > gpurun_out/ensdepth_${x}_$rep.json 2>/dev/null
    python -c "import json; d=json.load(open('gpurun_out/ensdepth_${x}_$rep.json'))['secondary']['2des']; print('depth=$x', d['ms_per_grid'], d['shard_1of8']['ms_per_grid'], d['shard_1of8']['event_ms_per_grid'], d['shard_1of8']['roofline']['frac'])"
  done
done
