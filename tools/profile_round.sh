#!/bin/bash
# Profiling recipe run on the GPU box (gpurun), in two calls so that no call runs long without output:
#   bash tools/profile_round.sh TAG stats   kernel-trace stats of the full bench, MFMA clock microbench,
#                                           byte-count calibration passes
#   bash tools/profile_round.sh TAG pmc     separate FETCH_SIZE / WRITE_SIZE passes (never combined with
#                                           other traces) of the default bench and of the general Lindblad kernel
# Output under gpurun_out/TAG.
set -e
TAG=${1:-prof}
PART=${2:-stats}
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
# a cooperative launch makes rocprofv3 segfault at process exit, with --pmc and (seen in r04) with --kernel-trace
# too, after the output is written (profiles/r04/pmc_crash/SUMMARY.md): every profiled run takes the plain launch
# of the banded DEOM and single-trajectory Lindblad kernels (same kernels, same residency)
export QD_COOP_LAUNCH=0
if [ "$PART" = stats ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 $R/bench.py --steps 50 --warmup 5 --no-cpu --no-deom-corr4 > $OUT/stats.log 2>&1
  rm -f $OUT/stats/run_kernel_trace.csv   # per-dispatch rows (tens of MB); the per-kernel summary stays
  timeout -k 10 60 $R/tools/mfma_f64_peak > $OUT/mfma_f64_peak.log 2>&1
  timeout -k 10 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/calib_fetch -o run -- $R/tools/pmc_calib > $OUT/calib_fetch.log 2>&1
  timeout -k 10 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/calib_write -o run -- $R/tools/pmc_calib > $OUT/calib_write.log 2>&1
else
  # without the banded-DEOM leg: the profiler's dispatch callback can read past a 1 MiB kernel-argument pool chunk
  # and segfault, likeliest on that leg's thousands of small launches (profiles/r05/runtime/pmc_crash/SUMMARY.md)
  timeout -k 10 250 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $R/bench.py --steps 20 --warmup 2 --no-cpu --no-deom-banded --no-deom-corr4 > $OUT/fetch.log 2>&1
  timeout -k 10 250 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $R/bench.py --steps 20 --warmup 2 --no-cpu --no-deom-banded --no-deom-corr4 > $OUT/write.log 2>&1
  timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/gfetch -o run -- python3 $R/bench.py --steps 20 --warmup 2 --no-cpu --general --no-2des --no-spo --no-deom --no-redfield > $OUT/gfetch.log 2>&1
  timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/gwrite -o run -- python3 $R/bench.py --steps 20 --warmup 2 --no-cpu --general --no-2des --no-spo --no-deom --no-redfield > $OUT/gwrite.log 2>&1
fi
