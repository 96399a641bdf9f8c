set -e
R=$PWD; OUT=$R/gpurun_out/prof7; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_redfield_response_gpu.py tests/test_deom_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu --no-spo --no-deom > $OUT/stats.log 2>&1
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu --no-spo --no-deom > $OUT/fetch.log 2>&1
