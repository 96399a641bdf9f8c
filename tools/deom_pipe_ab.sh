#!/bin/bash
# A/B of the software-pipelined persistent DEOM stage kernel (QD_DEOM_PIPE=1, default) against the stage kernels
# (QD_DEOM_PIPE=0: five-waves / wave-uniform instantiations), and its workgroups per class, on one box.
set -e
mkdir -p gpurun_out
for rep in 1 2; do
  for cfg in "QD_DEOM_PIPE=1" "QD_DEOM_PIPE=0" "QD_DEOM_PIPE_BPC=64" "QD_DEOM_PIPE_BPC=192"; do
    echo "== $cfg rep $rep"
    env $cfg timeout -k 10 120 python tools/deom_bench.py 64 72 128 2>/dev/null
  done
done
