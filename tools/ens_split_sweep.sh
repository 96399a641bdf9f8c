# 2DES fixed-t2 grid at one ensemble size over split counts / block sizes (QD_ENS_S, QD_ENS_BT)
set -e
M=${1:-4096}
OUT=gpurun_out/ens_sweep_$M; mkdir -p $OUT
for cfg in "0 0" "64 16" "64 32" "128 32" "128 64" "128 128"; do
  set -- $cfg
  bt=$1; s=$2
  QD_ENS_BT=$bt QD_ENS_S=$s timeout -k 10 120 python3 bench.py --steps 5 --warmup 2 --batch 8 --no-cpu --no-redfield \
    --no-spo --no-spo3 --no-superop --no-deom --t2 0 --ens $M --ens-reps 50 > $OUT/bt${bt}_s${s}.json
  python3 -c "import json,sys; d=json.loads(open('$OUT/bt${bt}_s${s}.json').read().strip().splitlines()[-1])['secondary']['2des']; print('bt=$bt S=$s', d['ms_per_grid'], d['event_ms_per_grid'], d.get('shard_1of8',{}).get('ms_per_grid'))"
done
