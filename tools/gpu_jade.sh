# usage: bash tools/gpu_jade.sh TAG — the JADE GPU tests, then C5 end to end twice (warm-start time)
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_jade.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_jade_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_jade_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_jade_$TAG.log
for i in 1 2; do
  timeout -k 10 200 python3 tools/run_configs.py C5 > gpurun_out/c5_$TAG.$i.json 2> gpurun_out/c5_$TAG.$i.log || exit 1
  head -c 700 gpurun_out/c5_$TAG.$i.json; echo
done
