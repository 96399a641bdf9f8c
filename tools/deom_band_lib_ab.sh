# A/B of library builds on the banded one-hierarchy DEOM launch (tools/deom_band_sweep.py 400 256), three rounds:
#   bash tools/deom_band_lib_ab.sh libA.so libB.so ...   (paths relative to the repo root)
set -e
for rep in 1 2 3; do
  for lib in "$@"; do
    echo "== $lib rep $rep"
    QDYN_LIB=$lib timeout -k 10 120 python tools/deom_band_sweep.py 400 256 2>/dev/null
  done
done
