# usage: bash tools/gpu_r3h.sh TAG — whole -m gpu suite, C5 with the JADE breakdown (PICARD_TRACE),
# the one-rank-of-8 proxy twice with the default host team
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -60 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_$TAG.log
for i in 1 2; do
  PICARD_TRACE=1 timeout -k 10 200 python3 tools/run_configs.py C5 > gpurun_out/c5_$TAG.$i.json 2> gpurun_out/c5_$TAG.$i.log || exit 1
  grep "jade:" gpurun_out/c5_$TAG.$i.log; head -c 200 gpurun_out/c5_$TAG.$i.json; echo
done
bash tools/gpu_hostspikes.sh $TAG
