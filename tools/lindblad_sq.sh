# SQ / GRBM counters of the Lindblad leg alone (one pass, no trace): MFMA busy cycles against elapsed GPU cycles
set -e
R=$PWD
OUT=$R/gpurun_out/lindblad_sq
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_VALU_MFMA_MOPS_F64 GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT -o run -- python3 $R/bench.py --steps 20 --warmup 2 --no-cpu --no-2des --no-redfield --no-superop --no-spo --no-spo3 --no-deom > $OUT/run.log 2>&1
