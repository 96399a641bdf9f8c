# A/B of the DEOM batch layout (QD_DEOM_ADO_MAJOR=1: [nmax][B]; 0: [B][nmax]) on the bench hierarchy
# (L = 12, K = 5) at 64 and 256 hierarchies, alternating, two rounds.
set -e
for rep in 1 2; do
  for b in 64 256; do
    for m in 0 1; do
      QD_DEOM_ADO_MAJOR=$m timeout -k 10 120 python bench.py --steps 5 --warmup 1 --batch 4 --deom-batch $b --no-cpu \
        --no-2des --no-redfield --no-spo > gpurun_out/deom_layout_${m}_${b}_$rep.json 2>/dev/null
    done
  done
done
