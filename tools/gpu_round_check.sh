# Full GPU test suite, then the kernel-trace profiling pass (tools/profile_round.sh TAG stats).
#   bash tools/gpu_round_check.sh TAG
set -e
TAG=${1:-prof}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/gputest_$TAG.log 2>&1
bash tools/profile_round.sh $TAG stats
