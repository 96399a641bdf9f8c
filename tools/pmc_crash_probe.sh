#!/bin/bash
# reproduce the two `rocprofv3 --pmc` crashes of round 3 on the current tree and keep the logs.
#   1. the DEOM legs of bench.py WITH the tier-banded loopback leg (round 3 passed --no-deom-banded to every PMC pass)
#   2. the one-rank RCCL communicator: libqdyn's qd_comm_init and torch.distributed "nccl", without and with --pmc
# Each GPU step has its own time limit; the chain stops at the first failure (its log names it).
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/pmc_probe
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
step() { local name=$1; shift; echo "== $name: $*" >> $OUT/steps.log; "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "== $name rc=$rc" >> $OUT/steps.log; return $rc; }
step band_plain timeout -k 10 120 python3 $R/bench.py --steps 5 --warmup 1 --no-cpu --no-2des --no-spo --no-spo3 --no-redfield --no-superop --deom-steps 20 --detail $OUT/band_plain_detail.json &&
step band_pmc timeout -k 10 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/band_pmc -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu --no-2des --no-spo --no-spo3 --no-redfield --no-superop --deom-steps 20 --detail $OUT/band_pmc_detail.json &&
step qd_plain timeout -k 10 60 python3 $R/tools/rccl_pmc_probe.py qd &&
step torch_plain timeout -k 10 60 python3 $R/tools/rccl_pmc_probe.py torch &&
step qd_pmc timeout -k 10 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/qd_pmc -o run -- python3 $R/tools/rccl_pmc_probe.py qd &&
step torch_pmc timeout -k 10 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/torch_pmc -o run -- python3 $R/tools/rccl_pmc_probe.py torch
rc=$?
cat $OUT/steps.log
exit $rc
