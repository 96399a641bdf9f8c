set -e
for rep in 1 2 3; do for v in 0 1; do echo "== W5=$v rep $rep"; QD_DEOM_W5=$v timeout -k 10 120 python tools/deom_bench.py 32 64 128 2>/dev/null; done; done
