#!/bin/bash
# A/B of the workspace runtime: parked-buffer reuse (default build) against the call-scoped hipFreeAsync release
# (pyqed_amd/libqdyn_oldws.so: the previous qd_runtime.hip linked with the current objects), on the 2DES full grid and
# its 1/8 shard (tools/ens_grid_time.py), two alternating rounds, one box.
set -e
for rep in 1 2; do
  for lib in pyqed_amd/libqdyn.so pyqed_amd/libqdyn_oldws.so; do
    QDYN_LIB=$PWD/$lib timeout -k 10 120 python tools/ens_grid_time.py $(basename $lib .so) 2>/dev/null
  done
done
