set -e
mkdir -p gpurun_out/r05_h
for r in 1 2; do for v in base 384 512 768; do
  if [ $v = base ]; then unset QDYN_LIB; else export QDYN_LIB=$PWD/var/wg64_$v.so; fi
  timeout -k 10 120 python3 tools/ens_grid_time.py wg64_$v >> gpurun_out/r05_h/ens_ab.txt 2>/dev/null
done; done
cat gpurun_out/r05_h/ens_ab.txt
