#!/bin/bash
# Second probe call (see tools/pmc_crash_probe.sh): RCCL one-rank communicators without / with --pmc, then the
# banded-exit probe.  Stops at the first failure.
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/pmc_probe2
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
step() { local name=$1; shift; echo "== $name: $*" >> $OUT/steps.log; "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "== $name rc=$rc" >> $OUT/steps.log; return $rc; }
P="rocprofv3 --pmc FETCH_SIZE --output-format csv"
step qd_plain timeout -k 10 60 python3 $R/tools/rccl_pmc_probe.py qd &&
step torch_plain timeout -k 10 60 python3 $R/tools/rccl_pmc_probe.py torch &&
step launches_pmc timeout -k 10 120 $P -d $OUT/launches_pmc -o run -- python3 $R/tools/band_exit_probe.py launches 30000 &&
step qd_pmc timeout -k 10 60 $P -d $OUT/qd_pmc -o run -- python3 $R/tools/rccl_pmc_probe.py qd &&
step torch_pmc timeout -k 10 60 $P -d $OUT/torch_pmc -o run -- python3 $R/tools/rccl_pmc_probe.py torch
rc=$?
cat $OUT/steps.log
exit $rc
