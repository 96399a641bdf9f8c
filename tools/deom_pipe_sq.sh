#!/bin/bash
# SQ instruction / cycle counters of the batched DEOM stage kernels at 64 hierarchies: the software-pipelined kernel
# (QD_DEOM_PIPE=1) and the five-waves stage kernel (=0), one --pmc pass each (no trace).  Output under
# gpurun_out/deom_pipe_sq; VALU pipe occupancy = 4 x SQ_INSTS_VALU / (1024 SIMDs x GRBM_GUI_ACTIVE / 8).
set -e
R=$PWD
OUT=$R/gpurun_out/deom_pipe_sq
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for a in 1 0; do
  QD_DEOM_PIPE=$a DEOM_STEPS=3 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq_$a -o run -- python3 $R/tools/deom_bench.py 64 > $OUT/sq_$a.log 2>&1
done
