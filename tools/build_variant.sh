# Build a library variant with one source recompiled under extra flags:
#   bash tools/build_variant.sh <out.so> <source.hip> "-DFOO=1 ..."
# (the other objects come from pyqed_amd/csrc/build/, i.e. the current default build)
set -e
out=$1; src=$2; flags=$3
cd pyqed_amd/csrc
mkdir -p build_v
obj=build_v/$(basename $src .hip)_$(basename $out .so).o
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $flags -c $src -o $obj
objs=$(ls build/*.o | grep -v "build/$(basename $src .hip).o")
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../../$out $objs $obj -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo built $out
