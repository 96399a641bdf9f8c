# A/B of the DEOM group kernel's XCD block classes (QD_DEOM_XCD: 0 = flat numbering, 1 = all hierarchies on one
# block class, unset = 8 classes when 8 | B) on the bench hierarchy (L = 12, K = 5) at 1, 64 and 256 hierarchies.
set -e
for rep in 1 2; do
  for b in 64 256; do
    for x in 0 1 def; do
      if [ $x = def ]; then unset QD_DEOM_XCD; else export QD_DEOM_XCD=$x; fi
      timeout -k 10 120 python bench.py --steps 5 --warmup 1 --batch 4 --deom-batch $b --no-cpu \
        --no-2des --no-redfield --no-spo --no-superop > gpurun_out/deom_xcd_${x}_${b}_$rep.json 2>/dev/null
    done
  done
done
unset QD_DEOM_XCD
