#!/bin/bash
# Round-end evidence on one GPU box, each step under its own time limit, stopping at the first failure:
# the GPU test suite, smoke(), the driver's bench command, and the profile passes (kernel trace + PMC bytes).
set -e
TAG=${1:-r04_final}
mkdir -p gpurun_out/$TAG
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/gputest.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$TAG/smoke.log 2>&1
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 --detail gpurun_out/$TAG/bench_detail.json > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
bash tools/profile_round.sh prof_$TAG stats
bash tools/profile_round.sh prof_$TAG pmc
tail -2 gpurun_out/$TAG/gputest.log; tail -1 gpurun_out/$TAG/smoke.log
