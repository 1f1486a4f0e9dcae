# usage: bash tools/gpu_tests_configs.sh TAG [configs...] — gpu tests then BASELINE configs end to end
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_$TAG.log
PICARD_TRACE=1 bash tools/gpu_configs.sh $TAG "$@" 2>&1 | grep -v "iter .* gnorm"
grep -h "jade:" gpurun_out/configs_${TAG}_*.err || true
