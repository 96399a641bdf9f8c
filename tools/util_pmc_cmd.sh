# Utilisation PMC pass + kernel-trace stats of an arbitrary python command (args), summarised per kernel
# (tools/util_summary.py) with the average durations alongside.  Output under gpurun_out/$1.
R=$PWD
OUT=$R/gpurun_out/$1
shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export QD_COOP_LAUNCH=0
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/t -o run -- python3 "$@" > $OUT/t.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/p -o run -- python3 "$@" > $OUT/p.log 2>&1 || exit $?
python3 $R/tools/util_summary.py $OUT/p/run_counter_collection.csv > $OUT/summary.txt
cp $OUT/t/run_kernel_stats.csv $OUT/kernel_stats.csv
rm -rf $OUT/p $OUT/t
