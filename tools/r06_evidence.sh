#!/bin/bash
# Round-6 evidence on one GPU box, each step under its own limit, stopping at the first failure:
#   part 1: the GPU test suite, smoke(), the driver's bench command, the kernel-trace stats pass (+ MFMA clock bench,
#           PMC calibration passes)       bash tools/r06_evidence.sh TAG 1
#   part 2: the separate FETCH_SIZE / WRITE_SIZE passes (tools/profile_round.sh pmc)
#                                         bash tools/r06_evidence.sh TAG 2
set -e
TAG=${1:-r06_final}
PART=${2:-1}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ "$PART" = 1 ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rs > $OUT/gputest.log 2>&1 || { tail -40 $OUT/gputest.log; exit 1; }
  tail -2 $OUT/gputest.log
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
  tail -1 $OUT/smoke.log
  timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --detail $OUT/bench_detail.json > $OUT/bench.json 2> $OUT/bench.err
  head -c 600 $OUT/bench.json; echo
  bash tools/profile_round.sh prof_$TAG stats
  echo "stats ok"
else
  bash tools/profile_round.sh prof_$TAG pmc
  echo "pmc ok"
fi
