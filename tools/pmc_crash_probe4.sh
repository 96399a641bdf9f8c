#!/bin/bash
# Fourth probe call: the persistent banded DEOM kernel alone, then followed by the loopback bands, under --pmc.
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/pmc_probe4
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
step() { local name=$1; shift; echo "== $name: $*" >> $OUT/steps.log; "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "== $name rc=$rc" >> $OUT/steps.log; return $rc; }
P="rocprofv3 --pmc FETCH_SIZE --output-format csv"
step persist_pmc timeout -k 10 120 $P -d $OUT/persist_pmc -o run -- python3 $R/tools/band_exit_probe.py persist &&
step both_pmc timeout -k 10 120 $P -d $OUT/both_pmc -o run -- python3 $R/tools/band_exit_probe.py both
rc=$?
cat $OUT/steps.log
exit $rc
