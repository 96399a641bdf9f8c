# A/B of the Lindblad paths on one box: the default library and each var/libqdyn_<name>.so given as arguments,
# alternating twice.  Output under gpurun_out/$1.
set -e
OUT=gpurun_out/$1
shift
mkdir -p $OUT
for i in 1 2; do
  for v in "$@"; do
    QDYN_LIB=$PWD/var/libqdyn_$v.so timeout -k 10 200 python3 tools/glf_ab.py > $OUT/${v}_$i.log 2>&1
  done
  timeout -k 10 200 python3 tools/glf_ab.py > $OUT/new_$i.log 2>&1
done
