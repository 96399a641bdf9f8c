# A/B of library builds on the Redfield bench leg: bash tools/redfield_ab.sh libA.so libB.so ...  (2 alternating rounds)
set -e
for rep in 1 2; do
  for lib in "$@"; do
    QDYN_LIB=$lib timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu --no-2des --no-spo --no-deom \
      --no-superop --no-spo3 > gpurun_out/rab_$(basename $lib .so)_$rep.json 2>/dev/null
    python -c "import json; d=json.load(open('gpurun_out/rab_$(basename $lib .so)_$rep.json')); r=d['secondary']['redfield']; print('$lib', 'lindblad', d['value'], 'redfield', r['value'], r['roofline']['frac'])"
  done
done
