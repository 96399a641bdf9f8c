# FETCH_SIZE / WRITE_SIZE passes (separate runs) of the bench's 2DES legs alone (fixed-t2 grid + waiting-time scan)
set -e
R=$PWD
OUT=$R/gpurun_out/prof_2des
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
A="--steps 2 --warmup 1 --batch 4 --no-cpu --no-redfield --no-superop --no-spo --no-spo3 --no-deom"
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $R/bench.py $A > $OUT/fetch.log 2>&1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $R/bench.py $A > $OUT/write.log 2>&1
