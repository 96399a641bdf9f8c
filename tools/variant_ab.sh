# A/B of library variants on the Lindblad + 2DES bench legs: bash tools/variant_ab.sh libA.so libB.so ...
set -e
for rep in 1 2; do
  for lib in "$@"; do
    QDYN_LIB=pyqed_amd/$lib timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-spo --no-deom --no-cpu --no-redfield --ens-reps 5 --t2-reps 2 > gpurun_out/ab_${lib%.so}_$rep.log 2>&1
  done
done
