# Kernel trace of the SPO legs of bench.py (SPO2 single + 64-wavepacket batch, SPO3 64^3 x 2). Output under
# gpurun_out/prof_spo.
set -e
R=$PWD
OUT=$R/gpurun_out/prof_spo
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
[ "$1" = pmc ] || timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 $R/bench.py --steps 5 --warmup 1 --batch 4 --no-cpu --no-2des --no-redfield --no-superop --no-deom > $OUT/bench.log 2>&1
if [ "$1" = pmc ]; then
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o run -- python3 $R/bench.py --steps 2 --warmup 1 --batch 4 --no-cpu --no-2des --no-redfield --no-superop --no-deom --no-spo3 --spo-steps 50 > $OUT/sq.log 2>&1
fi
