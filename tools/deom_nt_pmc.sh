# DEOM at 256 hierarchies: FETCH_SIZE and WRITE_SIZE per stage launch with plain (QD_DEOM_NT=0) and non-temporal
# (QD_DEOM_NT=1) RK4 state accesses; separate rocprofv3 passes, output under gpurun_out/deom_nt_pmc.
set -e
R=$PWD
OUT=$R/gpurun_out/deom_nt_pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for x in 0 1; do
  for c in FETCH_SIZE WRITE_SIZE; do
    QD_DEOM_NT=$x DEOM_STEPS=3 timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $OUT/${c}_$x -o run -- python3 $R/tools/deom_bench.py 256 > $OUT/${c}_$x.log 2>&1
  done
done
