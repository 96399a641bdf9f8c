# One utilisation PMC pass over the bench (no banded / Krylov legs), summarised per kernel by tools/util_summary.py.
# Output: gpurun_out/$1/summary.txt (the per-dispatch CSV is deleted).
R=$PWD
OUT=$R/gpurun_out/${1:-util_pmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export QD_COOP_LAUNCH=0
timeout -k 10 250 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/p -o run -- python3 $R/bench.py --steps 20 --warmup 2 --no-cpu --no-deom-banded --no-deom-corr4 > $OUT/p.log 2>&1
rc=$?
echo "rc=$rc"
[ $rc -eq 0 ] && python3 $R/tools/util_summary.py $OUT/p/run_counter_collection.csv > $OUT/summary.txt && rm -rf $OUT/p
exit $rc
