#!/bin/bash
# SPO3 block-width sweep: mid (y) pass QD_SPO3_MID_C x x-pass QD_SPO3_COL_C, + kernel trace of the default.
set -e
mkdir -p gpurun_out/spo3c
timeout -k 10 300 python -u -m pytest tests/test_spo_gpu.py -x -q --timeout 120 --timeout-method thread -k spo3 > gpurun_out/spo3c/tests.log 2>&1
for m in auto 8; do
  for c in fast 0 2 4 8; do
    if [ "$m" = auto ]; then unset QD_SPO3_MID_C; else export QD_SPO3_MID_C=$m; fi
    if [ "$c" = fast ]; then unset QD_SPO3_COL_C; else export QD_SPO3_COL_C=$c; fi
    timeout -k 10 120 python -u tools/spo3_bench.py >> gpurun_out/spo3c/sweep.log 2>&1
  done
done
unset QD_SPO3_MID_C QD_SPO3_COL_C
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/spo3c/prof -o spo3 -- python3 $GRAFT_REPO_ROOT/tools/spo3_bench.py > $GRAFT_REPO_ROOT/gpurun_out/spo3c/prof.log 2>&1
