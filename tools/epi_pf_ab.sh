# A/B of the Hermitian Lindblad epilogue: pipelined rho / acc loads (default build, GLF_EPI_PF=4) vs the chunked
# loads (pyqed_amd/libqdyn_pf0.so, GLF_EPI_PF=0); Lindblad leg of bench.py only, alternating, 3 rounds
set -e
for r in 1 2 3; do
  for lib in pyqed_amd/libqdyn.so pyqed_amd/libqdyn_pf0.so; do
    QDYN_LIB=$lib timeout -k 10 120 python bench.py --no-cpu --no-2des --no-spo --no-spo3 --no-deom --no-superop \
      --no-redfield --steps 50 > /tmp/ab.json 2>/dev/null
    python - "$lib" <<'PY'
import json, sys
d = json.loads(open('/tmp/ab.json').read().strip().splitlines()[-1])
print(sys.argv[1], d["value"], d["roofline"]["frac"], d["roofline"]["launch_ms"], d["batch_sweep"]["64"]["dm_steps_per_s"])
PY
  done
done
