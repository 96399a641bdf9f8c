# Lindblad persistent kernel: phase offset of every other workgroup per XCD (QD_STAGGER_US) vs none
set -e
for rep in 1 2; do
for s in 0 20 45 90; do
  QD_STAGGER_US=$s timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu --no-2des --no-spo --no-deom \
    --no-redfield --no-superop > gpurun_out/stag_${s}_$rep.json 2>/dev/null
  python -c "import json; d=json.load(open('gpurun_out/stag_${s}_$rep.json')); print('stagger $s us', d['value'], d['roofline']['frac'])"
done
done
