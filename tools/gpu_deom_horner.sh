set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_deom_gpu.py tests/test_deom_banded_gpu.py tests/test_deom_large_gpu.py tests/test_deom_multirank_gpu.py tests/test_heom_chain_gpu.py > gpurun_out/t_deom_horner.log 2>&1
for h in 0 1 0 1; do QD_DEOM_HORNER=$h timeout -k 10 120 python tools/deom_bench.py 16 64 256 >> gpurun_out/deom_horner_ab.txt 2>&1; echo "^ horner=$h" >> gpurun_out/deom_horner_ab.txt; done
QDYN_LIB=pyqed_amd/libqdyn_timing.so timeout -k 10 200 python tools/phase_timing.py > gpurun_out/phase_r03h.txt 2>&1
