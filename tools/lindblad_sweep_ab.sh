# A/B of library builds on the Lindblad leg incl. its batch sweep (B = 1, 64, 256), two alternating rounds:
#   bash tools/lindblad_sweep_ab.sh libA.so libB.so ...   (paths relative to the repo root)
set -e
for rep in 1 2; do
  for lib in "$@"; do
    QDYN_LIB=$lib timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu --no-2des --no-spo --no-deom \
      --no-redfield --no-superop --no-spo3 --no-deom-banded 2>/dev/null | grep '^{' > gpurun_out/lsab.json
    python -c "import json; d=json.load(open('gpurun_out/lsab.json')); b=d['batch_sweep']; print('$lib', 'B256', d['value'], 'B64', b['64']['dm_steps_per_s'], b['64']['roofline']['frac'], 'B1', b['1']['dm_steps_per_s'])"
  done
done
