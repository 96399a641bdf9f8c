#!/bin/bash
# Round-5 check on one GPU box: the GPU test suite, the driver's bench command, and the full-bench PMC pass that
# segfaulted with round 4's parked scratch, each under its own limit, stopping at the first
# failure.  Output under gpurun_out/TAG.
set -e
TAG=${1:-r05_check}
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $OUT/gputest.log 2>&1 || { tail -30 $OUT/gputest.log; exit 1; }
tail -2 $OUT/gputest.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --detail $OUT/bench_detail.json > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json | head -c 1500; echo
cd /tmp && export TMPDIR=/tmp
export QD_COOP_LAUNCH=0 BENCH_MAPS=$OUT/maps.txt
timeout -k 10 250 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $R/bench.py --steps 20 --warmup 2 --no-cpu --detail $OUT/fetch_detail.json > $OUT/fetch.log 2>&1
echo "pmc pass ok"
