# A/B of an environment switch on the Lindblad leg incl. its batch sweep, two alternating rounds:
#   bash tools/lindblad_env_ab.sh VAR value_a value_b ...
set -e
var=$1; shift
for rep in 1 2; do
  for v in "$@"; do
    env $var=$v timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu --no-2des --no-spo --no-deom \
      --no-redfield --no-superop --no-spo3 --no-deom-banded 2>/dev/null | grep '^{' > gpurun_out/leab.json
    python -c "import json; d=json.load(open('gpurun_out/leab.json')); b=d['batch_sweep']; print('$var=$v', 'B256', d['value'], 'B64', b['64']['dm_steps_per_s'], b['64']['roofline']['frac'], 'B1', b['1']['dm_steps_per_s'])"
  done
done
