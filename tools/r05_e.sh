set -e
mkdir -p gpurun_out/r05_e
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 200 --timeout-method thread > gpurun_out/r05_e/gputest.log 2>&1 || { tail -40 gpurun_out/r05_e/gputest.log; exit 1; }
tail -2 gpurun_out/r05_e/gputest.log
for v in base new base new; do
  if [ $v = base ]; then export QDYN_LIB=$PWD/var/ens_base.so; else unset QDYN_LIB; fi
  timeout -k 10 120 python3 tools/ens_grid_time.py $v >> gpurun_out/r05_e/ens_ab.txt 2>/dev/null
done
cat gpurun_out/r05_e/ens_ab.txt
