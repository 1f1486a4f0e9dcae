# usage: bash tools/gpu_configs.sh TAG — gpu tests, then BASELINE configs C2/C4/C5 end to end
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_$TAG.log
for c in C2 C4 C5; do
  timeout -k 10 240 python tools/run_configs.py $c >> gpurun_out/configs_$TAG.jsonl 2> gpurun_out/configs_${TAG}_$c.err || { echo "$c failed/timeout"; tail -5 gpurun_out/configs_${TAG}_$c.err; exit 1; }
  tail -1 gpurun_out/configs_$TAG.jsonl | cut -c1-400
done
