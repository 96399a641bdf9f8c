# DEOM ADO-major batches: hierarchies of an XCD class walked in chunks of 16 (default where classes are larger)
# vs all at once (QD_DEOM_BCHUNK=0) vs chunks of 8; tools/deom_bench.py at 256 / 512 hierarchies, three rounds.
set -e
for rep in 1 2 3; do
  for v in 0 16 8; do
    QD_DEOM_BCHUNK=$v timeout -k 10 120 python tools/deom_bench.py 256 512 | sed "s/^/QD_DEOM_BCHUNK=$v $rep /"
  done
done
