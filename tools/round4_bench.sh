#!/bin/bash
# Round-4 check: the Lindblad / SPO-build GPU tests touched since the last full run, then the full bench line.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_lindblad_gpu.py tests/test_spo_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r4_tests.log 2>&1; rc=$?; tail -4 gpurun_out/r4_tests.log
[ $rc -eq 0 ] || exit $rc
TAG=${1:-r04b}
timeout -k 10 700 python3 bench.py --detail gpurun_out/bench_${TAG}_detail.json > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err; rc=$?
tail -c 4000 gpurun_out/bench_${TAG}.json
exit $rc
