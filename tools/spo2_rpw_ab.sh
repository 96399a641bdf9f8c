# SPO2 64-wavepacket batch: one vs two members per wave in the row pass (QD_SPO_RPW), with 4 or 2 waves per
# workgroup (QD_SPO_ROWWAVE); bench SPO2 leg only, three alternating rounds.
set -e
for rep in 1 2 3; do
  for v in "QD_SPO_RPW=1" "QD_SPO_RPW=2" "QD_SPO_RPW=2 QD_SPO_ROWWAVE=2"; do
    tag=$(echo $v | tr ' =' '__')
    env $v timeout -k 10 120 python bench.py --steps 2 --warmup 1 --batch 4 --no-cpu --no-2des --no-redfield \
      --no-superop --no-spo3 --no-deom > gpurun_out/rpw_${tag}_$rep.json 2>/dev/null
    python -c "import json; d=json.load(open('gpurun_out/rpw_${tag}_$rep.json'))['secondary']['spo2']; b=d['batched']; print('$v', d['value'], b['wavepacket_steps_per_s'], b['roofline']['frac'])"
  done
done
