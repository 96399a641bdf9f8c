# A/B of library builds on the Lindblad bench leg: bash tools/lib_ab.sh libA.so libB.so ...  (2 alternating rounds)
set -e
for rep in 1 2; do
  for lib in "$@"; do
    QDYN_LIB=$lib timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu --no-2des --no-spo --no-deom \
      --no-redfield --no-superop --no-spo3 > gpurun_out/ab_$(basename $lib .so)_$rep.json 2>/dev/null
    python -c "import json; d=json.load(open('gpurun_out/ab_$(basename $lib .so)_$rep.json')); print('$lib', d['value'], d['roofline']['frac'], d['ms_per_step'])"
  done
done
