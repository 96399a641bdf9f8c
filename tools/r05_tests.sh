#!/bin/bash
# GPU test suite (up to 10 failures reported), then optional extra commands given as arguments.  Output under
# gpurun_out/TAG.
TAG=${1:-r05_tests}
shift
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 200 --timeout-method thread > $OUT/gputest.log 2>&1
rc=$?
tail -40 $OUT/gputest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for cmd in "$@"; do
  echo "== $cmd"
  eval "timeout -k 10 300 $cmd" || exit $?
done
exit $rc
