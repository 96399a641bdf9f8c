#!/bin/bash
# Round-2 closing profile of the default bench (run on the GPU box in two calls):
#   bash tools/profile_r02b.sh stats   kernel-trace --stats of `python bench.py` (the driver's command) + the
#                                      FETCH_SIZE / WRITE_SIZE byte calibration passes (tools/pmc_calib)
#   bash tools/profile_r02b.sh pmc     separate FETCH_SIZE and WRITE_SIZE passes of `bench.py --steps 20 --warmup 2
#                                      --no-cpu` (no other counter or trace in the same run)
set -e
PART=${1:-stats}
R=$PWD
OUT=$R/gpurun_out/${PROF_TAG:-prof_r02b}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
if [ "$PART" = stats ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 $R/bench.py > $OUT/stats.log 2>&1
  timeout -k 10 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/calib_fetch -o run -- $R/tools/pmc_calib > $OUT/calib_fetch.log 2>&1
  timeout -k 10 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/calib_write -o run -- $R/tools/pmc_calib > $OUT/calib_write.log 2>&1
else
  timeout -k 10 280 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $R/bench.py --steps 20 --warmup 2 --no-cpu > $OUT/fetch.log 2>&1
  timeout -k 10 280 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $R/bench.py --steps 20 --warmup 2 --no-cpu > $OUT/write.log 2>&1
fi
