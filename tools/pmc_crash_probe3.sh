#!/bin/bash
# Third probe call (see tools/pmc_crash_probe.sh): the bench's RCCL leg under --pmc, then the banded loopback alone
# under --pmc with libqdyn's pool trimmed before exit (qd_shutdown) and with a plain exit.  Stops at the first failure.
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/pmc_probe3
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
step() { local name=$1; shift; echo "== $name: $*" >> $OUT/steps.log; "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "== $name rc=$rc" >> $OUT/steps.log; return $rc; }
P="rocprofv3 --pmc FETCH_SIZE --output-format csv"
step bench_reduce_pmc timeout -k 10 200 $P -d $OUT/bench_reduce_pmc -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu --no-spo --no-spo3 --no-redfield --no-superop --no-deom --t2 0 --ens-reps 3 --detail $OUT/bench_reduce_detail.json &&
step band_shutdown_pmc timeout -k 10 120 $P -d $OUT/band_shutdown_pmc -o run -- python3 $R/tools/band_exit_probe.py shutdown &&
step band_plain_pmc timeout -k 10 120 $P -d $OUT/band_plain_pmc -o run -- python3 $R/tools/band_exit_probe.py plain
rc=$?
cat $OUT/steps.log
exit $rc
