# A/B of the Z-operand block grouping (QD_Z_MINBLOCKS: minimum number of member blocks; 0 = LDS-sized groups)
set -e
for mb in 0 512 1024 2048; do  # 0 = LDS-sized groups only
  for m in 4096 32768; do
    QD_Z_MINBLOCKS=$mb timeout -k 10 120 python bench.py --steps 5 --warmup 2 --batch 8 --no-cpu --no-redfield \
      --no-spo --no-deom --ens $m > gpurun_out/zb_${mb}_$m.json 2>/dev/null
  done
done
