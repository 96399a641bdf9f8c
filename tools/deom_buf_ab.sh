#!/bin/bash
# A/B of the pipelined DEOM stage kernel's buffer-load gathers (default build) against the 64-bit global-address
# form (pyqed_amd/libqdyn_nobuf.so, built at the commit that added the gathers with tools/build_variant.sh ...
# deom.hip -DDEOM_PIPE_BUF=0; the switch was removed once measured), alternating, one box.
set -e
for rep in 1 2; do
  for lib in pyqed_amd/libqdyn.so pyqed_amd/libqdyn_nobuf.so; do
    echo "== $lib rep $rep"
    QDYN_LIB=$PWD/$lib timeout -k 10 120 python tools/deom_bench.py 64 72 128 2>/dev/null
  done
done
