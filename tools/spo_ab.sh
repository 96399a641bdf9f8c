# A/B of the any-grid SPO passes: the default library against var/libqdyn_base.so (same box, alternating).
# Output under gpurun_out/$1.
set -e
OUT=gpurun_out/${1:-spo_ab}
mkdir -p $OUT
for i in 1 2; do
  QDYN_LIB=$PWD/var/libqdyn_base.so timeout -k 10 200 python3 tools/spo_any_bench.py ${2:-200,500,1000} ${3:-all} > $OUT/base_$i.log 2>&1
  timeout -k 10 200 python3 tools/spo_any_bench.py ${2:-200,500,1000} ${3:-all} > $OUT/new_$i.log 2>&1
done
