# DEOM group kernel: non-temporal RK4 state accesses (QD_DEOM_NT=1) vs plain (QD_DEOM_NT=0); tools/deom_bench.py
# event timing at 64/128/256 hierarchies, three alternating rounds.
set -e
for rep in 1 2 3; do
  for nt in 0 1; do
    QD_DEOM_NT=$nt timeout -k 10 120 python tools/deom_bench.py 64 128 256 | sed "s/^/QD_DEOM_NT=$nt $rep /"
  done
done
