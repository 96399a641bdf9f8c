# A/B of the Z-operand block grouping (QD_Z_MINBLOCKS: minimum number of member blocks; 0 = LDS-sized groups),
# 2DES leg only at the bench ensemble (32,768) and one rank's shard (4,096): ms per grid, two rounds.
set -e
for rep in 1 2; do
  for mb in 1024 4096 8192 16384; do
    QD_Z_MINBLOCKS=$mb timeout -k 10 120 python bench.py --steps 2 --warmup 1 --batch 4 --no-cpu --no-redfield \
      --no-superop --no-spo --no-spo3 --no-deom --t2 0 > gpurun_out/zb_${mb}_$rep.json 2>/dev/null
    python -c "import json; d=json.load(open('gpurun_out/zb_${mb}_$rep.json'))['secondary']['2des']; print('minblocks=$mb', d['ms_per_grid'], d['event_ms_per_grid'], d['shard_1of8']['ms_per_grid'])"
  done
done
