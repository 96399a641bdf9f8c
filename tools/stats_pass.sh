#!/bin/bash
# One rocprofv3 kernel-trace/stats pass of the full bench on the GPU box: gpurun_out/$1/{stats,stats.log}
set -e
TAG=${1:-stats}
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 $R/bench.py --steps 50 --warmup 5 --no-cpu > $OUT/stats.log 2>&1
