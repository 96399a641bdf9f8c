# One DEOM hierarchy (6188 ADOs): every stage block on one XCD (QD_DEOM_XCD=1: the state stays in one L2) vs the
# flat numbering over all 8 XCDs (QD_DEOM_XCD=0, the default for B = 1); tpb 64 / 256; event-timed, two rounds
set -e
for rep in 1 2; do
  for x in 0 1; do
    for t in 64 256; do
      QD_DEOM_XCD=$x QD_DEOM_TPB=$t DEOM_STEPS=200 timeout -k 10 120 python tools/deom_bench.py 1 | sed "s/^/xcd=$x tpb=$t /"
    done
  done
done
