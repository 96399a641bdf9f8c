# A/B of the single-trajectory launch: var/libqdyn_base.so against the default library (tools/glf_single_bench.py,
# alternating twice on one box).  Output under gpurun_out/$1.
set -e
OUT=gpurun_out/${1:-glf_single_ab}
mkdir -p $OUT
for i in 1 2; do
  QDYN_LIB=$PWD/var/libqdyn_base.so timeout -k 10 200 python3 tools/glf_single_bench.py 300 > $OUT/base_$i.log 2>&1
  timeout -k 10 200 python3 tools/glf_single_bench.py 300 > $OUT/new_$i.log 2>&1
done
