# kernel trace of the 2DES legs at a given ensemble size (per-rank shard of an N-GPU run)
set -e
R=$PWD; M=${1:-512}; OUT=$R/gpurun_out/p2d_$M; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 $R/bench.py --steps 5 --warmup 2 --batch 8 --no-cpu --no-redfield --no-spo --no-deom --ens $M > $OUT/bench.json 2> $OUT/err.log
