set -e
for s in 0 10 25 45 70; do
  QD_STAGGER_US=$s timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-2des --no-spo --no-deom --no-cpu > gpurun_out/stag_$s.log 2>&1
done
