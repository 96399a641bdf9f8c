# A/B of DEOM stage kernels on the bench hierarchy (L = 12, K = 5; 1 and 64 hierarchies):
#   bash tools/deom_ab.sh libA.so libB.so ...   (libraries under pyqed_amd/)
set -e
for rep in 1 2; do
  for lib in "$@"; do
    for tpb in 64 256; do
      QD_DEOM_TPB=$tpb QDYN_LIB=pyqed_amd/$lib timeout -k 10 120 python bench.py --steps 5 --warmup 1 --no-cpu \
        --no-2des --no-redfield --no-spo > gpurun_out/deom_ab_${lib%.so}_tpb${tpb}_$rep.log 2>&1
    done
  done
done
