#!/bin/bash
# Fifth probe call: is the exit-time SIGSEGV under --pmc the cooperative launch?  The persistent banded DEOM run with a
# plain launch (QD_DEOM_BAND_COOP=0), then a trivial HIP program: plain launch, then cooperative launch.
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/pmc_probe5
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
step() { local name=$1; shift; echo "== $name: $*" >> $OUT/steps.log; "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "== $name rc=$rc" >> $OUT/steps.log; return $rc; }
P="rocprofv3 --pmc FETCH_SIZE --output-format csv"
export QD_DEOM_BAND_COOP=0
step persist_plainlaunch_pmc timeout -k 10 120 $P -d $OUT/persist_plainlaunch_pmc -o run -- python3 $R/tools/band_exit_probe.py persist &&
step trivial_plain_pmc timeout -k 10 60 $P -d $OUT/trivial_plain_pmc -o run -- $R/tools/coop_pmc_probe 0 &&
step trivial_coop_nopmc timeout -k 10 60 $R/tools/coop_pmc_probe 1 &&
step trivial_coop_pmc timeout -k 10 60 $P -d $OUT/trivial_coop_pmc -o run -- $R/tools/coop_pmc_probe 1
rc=$?
cat $OUT/steps.log
exit $rc
