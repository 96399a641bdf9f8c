# A/B of the single-trajectory launch on one box: the default library and each var/libqdyn_<name>.so given as
# arguments (default: base), alternating twice (tools/glf_single_bench.py).  Output under gpurun_out/$1.
set -e
OUT=gpurun_out/${1:-glf_single_ab}
shift || true
VARIANTS=${@:-base}
mkdir -p $OUT
for i in 1 2; do
  for v in $VARIANTS; do
    QDYN_LIB=$PWD/var/libqdyn_$v.so timeout -k 10 200 python3 tools/glf_single_bench.py 300 > $OUT/${v}_$i.log 2>&1
  done
  timeout -k 10 200 python3 tools/glf_single_bench.py 300 > $OUT/new_$i.log 2>&1
done
