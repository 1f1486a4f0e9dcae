# usage: bash tools/gpu_rccl1.sh TAG — the one-rank RCCL tests, then C2 end to end with the
# per-iteration trace (PICARD_TRACE=1: step / eval / host ms per iteration)
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rccl.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_rccl_$TAG.log 2>&1 || { tail -60 gpurun_out/pytest_rccl_$TAG.log; exit 1; }
tail -8 gpurun_out/pytest_rccl_$TAG.log
for i in 1 2 3; do
  PICARD_TRACE=1 timeout -k 10 120 python3 tools/run_configs.py C2 > gpurun_out/c2_$TAG.$i.json 2> gpurun_out/c2_trace_$TAG.$i.log || exit 1
  head -c 400 gpurun_out/c2_$TAG.$i.json; echo
done
