# A/B of library variants on the Lindblad bench leg: bash tools/variant_ab.sh libA.so libB.so ...
set -e
for lib in "$@"; do
  for rep in 1 2; do
    QDYN_LIB=pyqed_amd/$lib timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-2des --no-spo --no-deom --no-cpu > gpurun_out/ab_${lib%.so}_$rep.log 2>&1
  done
done
