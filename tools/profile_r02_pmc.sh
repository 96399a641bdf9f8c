# Round-2 PMC passes (separate FETCH_SIZE / WRITE_SIZE runs of the default bench, nothing else collected with them).
set -e
R=$PWD
OUT=$R/gpurun_out/prof_r02
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 280 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $R/bench.py --steps 20 --warmup 2 --no-cpu > $OUT/fetch.log 2>&1
timeout -k 10 280 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $R/bench.py --steps 20 --warmup 2 --no-cpu > $OUT/write.log 2>&1
