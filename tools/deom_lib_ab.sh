# A/B of library builds on the batched DEOM stage launches (tools/deom_bench.py 16 64 256), two alternating rounds:
#   bash tools/deom_lib_ab.sh libA.so libB.so ...   (paths relative to the repo root)
set -e
for rep in 1 2; do
  for lib in "$@"; do
    echo "== $lib rep $rep"
    QDYN_LIB=$lib timeout -k 10 120 python tools/deom_bench.py 16 64 256 2>/dev/null
  done
done
