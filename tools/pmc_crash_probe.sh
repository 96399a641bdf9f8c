# PMC-pass crash probe (profiles/r05/runtime/pmc_crash.md), one GPU call: (1) the torch-only control under
# rocprofv3 --pmc FETCH_SIZE; (2) the bench's Lindblad + DEOM legs (incl. the banded loopback) under the same pass
# with the process map dumped per leg; the crash frames resolved on the box.  Stops GPU work at the first failure.
R=$PWD
O=$R/gpurun_out/${1:-pmc_dbg}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export QD_COOP_LAUNCH=0
BENCH_MAPS=$O/maps_torch.txt timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/torch -o run -- python3 $R/tools/pmc_torch_repro.py 6000 > $O/torch.log 2>&1
rc=$?
echo "torch control rc=$rc"; tail -2 $O/torch.log
if [ $rc -ne 0 ]; then python3 $R/tools/resolve_frames.py $O/torch.log $O/maps_torch.txt > $O/frames_torch.txt 2>&1; head -40 $O/frames_torch.txt; exit 0; fi
BENCH_MAPS=$O/maps.txt timeout -k 10 250 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $R/bench.py --steps 20 --warmup 2 --no-cpu --no-2des --no-spo --no-redfield --no-superop > $O/fetch.log 2>&1
rc=$?
echo "bench deom legs rc=$rc"; grep -v '^\s*@' $O/fetch.log | tail -3
if [ $rc -ne 0 ]; then python3 $R/tools/resolve_frames.py $O/fetch.log $O/maps.txt > $O/frames.txt 2>&1; head -40 $O/frames.txt; fi
exit 0
