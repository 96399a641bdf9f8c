# Kernel trace of the SPO legs of bench.py (SPO2 single + 64-wavepacket batch, SPO3 64^3 x 2). Output under
# gpurun_out/prof_spo.
set -e
R=$PWD
OUT=$R/gpurun_out/prof_spo
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 $R/bench.py --steps 5 --warmup 1 --batch 4 --no-cpu --no-2des --no-redfield --no-superop --no-deom > $OUT/bench.log 2>&1
