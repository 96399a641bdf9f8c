#!/bin/bash
# SPO any-grid check + timing (round 4): GPU tests of the SPO / FFT paths, spo_any_bench with and without the staged
# operators (QD_SPO_AUX), and a kernel trace of the 200 x 200 x 2 case.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_spo_anygrid_gpu.py tests/test_fft_gpu.py tests/test_spo_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/t_e.log 2>&1; rc=$?; tail -5 gpurun_out/t_e.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/spo_any_bench.py > gpurun_out/spo_any_e.txt 2>&1 || exit 1
timeout -k 10 200 python3 tools/glf_single_bench.py > gpurun_out/glf_single_e.txt 2>&1 || exit 1
QDYN_LIB=$PWD/pyqed_amd/libqdyn_timing.so timeout -k 10 120 python3 tools/glf_single_bench.py 50 > gpurun_out/glf_single_timing.txt 2>&1 || exit 1
QD_SPO_AUX=0 timeout -k 10 200 python3 tools/spo_any_bench.py 200,500 2d > gpurun_out/spo_any_e_noaux.txt 2>&1 || exit 1
cat gpurun_out/spo_any_e.txt gpurun_out/spo_any_e_noaux.txt gpurun_out/glf_single_e.txt
grep phase gpurun_out/glf_single_timing.txt
cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_spo200 -o run -- python3 $GRAFT_REPO_ROOT/tools/spo_any_bench.py 200 2d > $GRAFT_REPO_ROOT/gpurun_out/prof_spo200.log 2>&1
