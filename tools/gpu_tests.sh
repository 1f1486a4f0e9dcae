# usage: bash tools/gpu_tests.sh TAG [pytest-args] — GPU tests only (time-limited), log in gpurun_out/
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest ${@:-tests} -m gpu -x -q --timeout 300 --timeout-method thread --durations=10 \
  > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -80 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -25 gpurun_out/pytest_gpu_$TAG.log
