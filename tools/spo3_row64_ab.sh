# SPO3 64^3 x 2: 64-point register transforms for the z / y / x passes (QD_SPO_ROW64=1, default) vs the LDS
# Stockham kernels (=0); event-timed qd_spo3_run (32^3 / 64^3 / 128^3), then kernel traces at 64^3.
set -e
for rep in 1 2; do
  for f in 1 0; do
    QD_SPO_ROW64=$f SPO3_SIZES=32,64,128 timeout -k 10 120 python tools/spo3_bench.py | sed "s/^/row64=$f /"
  done
done
R=$PWD
cd /tmp && export TMPDIR=/tmp
for f in 1 0; do
  QD_SPO_ROW64=$f SPO3_SIZES=64 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $R/gpurun_out/spo3_r64_prof_$f -o run -- python3 $R/tools/spo3_bench.py > $R/gpurun_out/spo3_r64_prof_$f.log 2>&1
done
