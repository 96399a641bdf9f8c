set -e
mkdir -p gpurun_out/r05_d
for v in base var/xtab64_d1.so var/xtab64_d2.so base var/xtab64_d1.so var/xtab64_d2.so; do
  if [ $v = base ]; then unset QDYN_LIB; else export QDYN_LIB=$PWD/$v; fi
  timeout -k 10 120 python3 tools/ens_grid_time.py $v >> gpurun_out/r05_d/ens_ab.txt 2>/dev/null
done
unset QDYN_LIB
cat gpurun_out/r05_d/ens_ab.txt
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-cpu --no-2des --no-spo --no-spo3 --no-redfield --no-superop --detail gpurun_out/r05_d/deom_detail.json > gpurun_out/r05_d/deom.json 2> gpurun_out/r05_d/deom.err
python3 -c "
import json;d=json.load(open('gpurun_out/r05_d/deom_detail.json'))['secondary']['deom_banded']
for k,v in d.items():
  m=v['model_8gpu'];print(k, v['nmax'], 'band max us', m['max_band_stage_us'], 'single ms', m['one_gpu_unbanded_ms_per_step'], {x:m[x]['speedup'] for x in ('p2p_nolat','p2p_lat','allgather_lat')})
"
