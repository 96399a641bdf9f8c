set -e
mkdir -p gpurun_out/r05_c
timeout -k 10 300 python -u -m pytest tests/test_spo_anygrid_gpu.py tests/test_spo_gpu.py -q --timeout 200 --timeout-method thread > gpurun_out/r05_c/spo_tests.log 2>&1 || { tail -30 gpurun_out/r05_c/spo_tests.log; exit 1; }
tail -2 gpurun_out/r05_c/spo_tests.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05_c/ens -o run -- python3 $GRAFT_REPO_ROOT/tools/ens_grid_time.py base > $GRAFT_REPO_ROOT/gpurun_out/r05_c/ens.log 2>&1
cd $GRAFT_REPO_ROOT
tail -1 gpurun_out/r05_c/ens.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu --no-2des --no-spo --no-spo3 --no-redfield --no-superop --detail gpurun_out/r05_c/deom_detail.json > gpurun_out/r05_c/deom.json 2> gpurun_out/r05_c/deom.err
python3 -c "import json;d=json.load(open('gpurun_out/r05_c/deom_detail.json'));print(json.dumps(d['secondary']['deom_banded'],indent=0)[:3000])"
