# SQ instruction / cycle counters of the DEOM stage kernels (group kernel vs one-lane-per-ADO kernel) at 64 and
# 256 hierarchies; one --pmc pass per variant.  Output under gpurun_out/deom_sq.
set -e
R=$PWD
OUT=$R/gpurun_out/deom_sq
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for a in 0 1; do
  QD_DEOM_ADO2=$a DEOM_STEPS=3 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq_$a -o run -- python3 $R/tools/deom_bench.py 64 256 > $OUT/sq_$a.log 2>&1
done
