# usage: bash tools/gpu_check.sh TAG [pytest args …] — the given GPU tests (default: the whole
# -m gpu suite) under a per-step time limit; log in gpurun_out/check_TAG.log
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
ARGS=${@:-tests}
timeout -k 10 900 python -u -m pytest $ARGS -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/check_$TAG.log 2>&1 || { tail -60 gpurun_out/check_$TAG.log; exit 1; }
tail -3 gpurun_out/check_$TAG.log
