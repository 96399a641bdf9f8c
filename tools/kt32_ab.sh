# 2DES 1/8 shard and full grid with 32-wide K-tiles on 64-blocks (default) vs 16 (QD_ENS_KT32=0): bench 2DES leg.
set -e
for rep in 1 2; do
  for x in 1 0; do
    QD_ENS_KT32=$x timeout -k 10 150 python bench.py --steps 2 --warmup 1 --batch 4 --no-cpu --t2 0 --no-redfield \
      --no-superop --no-spo --no-spo3 --no-deom > gpurun_out/kt32_${x}_$rep.json 2>/dev/null
    python -c "import json; d=json.load(open('gpurun_out/kt32_${x}_$rep.json'))['secondary']['2des']; print('kt32=$x', d['ms_per_grid'], d['shard_1of8']['ms_per_grid'], d['shard_1of8']['roofline']['frac'])"
  done
done
