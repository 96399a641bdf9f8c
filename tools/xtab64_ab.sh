# 2DES 1/8 shard (4,096 members) and full grid with the generated A operand on 64-blocks (QD_ENS_XTAB64=1) vs
# the materialised X: bench 2DES leg only, two alternating rounds.
set -e
for rep in 1 2; do
  for x in 0 1; do
    QD_ENS_XTAB64=$x timeout -k 10 150 python bench.py --steps 2 --warmup 1 --batch 4 --no-cpu --t2 0 --no-redfield \
      --no-superop --no-spo --no-spo3 --no-deom > gpurun_out/xtab64_${x}_$rep.json 2>/dev/null
    python -c "import json; d=json.load(open('gpurun_out/xtab64_${x}_$rep.json'))['secondary']['2des']; print('xtab64=$x', d['ms_per_grid'], d['shard_1of8']['ms_per_grid'])"
  done
done
