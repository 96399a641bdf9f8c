# A/B of the SPO2 256x256x2 passes: register 16x16 FFT (QD_SPO_Q16=1, default) vs the LDS Stockham passes
set -e
for rep in 1 2; do
  for q in 0 1; do
    QD_SPO_Q16=$q timeout -k 10 120 python bench.py --steps 5 --warmup 1 --no-cpu --no-2des --no-redfield --no-deom \
      > gpurun_out/spo_ab_q${q}_$rep.log 2>&1
  done
done
