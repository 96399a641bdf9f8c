#!/bin/bash
# Profiling recipe run on the GPU box (gpurun): kernel-trace stats of the full bench and
# separate FETCH_SIZE / WRITE_SIZE passes (never combined with other traces), for the default
# (Hermitian) Lindblad kernel and the general one, plus the byte-count calibration kernels.
# Output under gpurun_out/$1.
set -e
TAG=${1:-prof}
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 $R/bench.py --steps 50 --warmup 5 --no-cpu > $OUT/stats.log 2>&1
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $R/bench.py --steps 20 --warmup 2 --no-cpu > $OUT/fetch.log 2>&1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $R/bench.py --steps 20 --warmup 2 --no-cpu > $OUT/write.log 2>&1
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/gfetch -o run -- python3 $R/bench.py --steps 20 --warmup 2 --no-cpu --general --no-2des --no-spo --no-deom > $OUT/gfetch.log 2>&1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/gwrite -o run -- python3 $R/bench.py --steps 20 --warmup 2 --no-cpu --general --no-2des --no-spo --no-deom > $OUT/gwrite.log 2>&1
timeout -k 10 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/calib_fetch -o run -- $R/tools/pmc_calib > $OUT/calib_fetch.log 2>&1
timeout -k 10 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/calib_write -o run -- $R/tools/pmc_calib > $OUT/calib_write.log 2>&1
