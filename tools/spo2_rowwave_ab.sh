# SPO2 64-wavepacket batch: row pass variants (QD_SPO_ROWMB=2 group kernel vs QD_SPO_ROWWAVE=2/4/8 wave-per-member
# kernel, default 4) and column tiles (QD_SPO_COLTILE=4 default / 8); bench SPO2 leg only, two alternating rounds.
set -e
for rep in 1 2; do
  for v in "QD_SPO_COLTILE=8" "QD_SPO_COLTILE=16" "QD_SPO_COLTILE=4"; do
    env $v timeout -k 10 120 python bench.py --steps 2 --warmup 1 --batch 4 --no-cpu --no-2des --no-redfield \
      --no-superop --no-spo3 --no-deom > gpurun_out/rowwave_${v}_$rep.json 2>/dev/null
    python -c "import json; d=json.load(open('gpurun_out/rowwave_${v}_$rep.json'))['secondary']['spo2']; b=d['batched']; print('$v', d['value'], b['wavepacket_steps_per_s'], b['roofline']['frac'])"
  done
done
