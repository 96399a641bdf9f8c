# DEOM group kernel: wave-uniform ADO with scalar index / prefactor loads (QD_DEOM_UNI default on where the XCD
# classes hold multiples of 16 hierarchies) vs per-group vector loads + DPP broadcasts (QD_DEOM_UNI=0);
# tools/deom_bench.py at 128 / 256 hierarchies (64: classes of 8, not eligible), three alternating rounds.
set -e
for rep in 1 2 3; do
  for v in 0 1; do
    QD_DEOM_UNI=$v timeout -k 10 120 python tools/deom_bench.py 64 128 256 | sed "s/^/QD_DEOM_UNI=$v $rep /"
  done
done
