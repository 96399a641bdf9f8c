# Build var/libqdyn_<name>.so: the library with extra compile definitions (A/B variants), e.g.
#   bash tools/build_variant.sh s10 -DSG_SLEEP_K=10 -DSG_SLEEP_Y=10
set -e
NAME=$1
shift
cd "$(dirname "$0")/../pyqed_amd/csrc"
mkdir -p ../../var/build_$NAME
objs=""
for f in *.hip; do
  o=../../var/build_$NAME/${f%.hip}.o
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 "$@" -c $f -o $o &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../../var/libqdyn_$NAME.so $objs -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -rf ../../var/build_$NAME
