# usage: bash tools/gpu_ab2.sh TAG KNOB — screen / int8 / group GPU tests, then screen timing with and
# without KNOB=1, then the C3 bench (no other configs) with and without it
TAG=$1; KNOB=$2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_screen32.py tests/test_gpu_int8.py tests/test_gpu_group.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_ab2_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_ab2_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_ab2_$TAG.log
timeout -k 10 120 python3 tools/bench_loss.py 128 2e7 5 auto || exit 1
env $KNOB=1 timeout -k 10 120 python3 tools/bench_loss.py 128 2e7 5 auto || exit 1
timeout -k 10 120 python3 tools/bench_loss.py 64 1e7 5 auto || exit 1
env $KNOB=1 timeout -k 10 120 python3 tools/bench_loss.py 64 1e7 5 auto || exit 1
timeout -k 10 400 python bench.py --cpu-baseline 0 --configs 0 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
python3 tools/bench_summary.py gpurun_out/bench_$TAG.json
env $KNOB=1 timeout -k 10 400 python bench.py --cpu-baseline 0 --configs 0 > gpurun_out/bench_${TAG}_off.json 2> gpurun_out/bench_${TAG}_off.err || { tail -20 gpurun_out/bench_${TAG}_off.err; exit 1; }
python3 tools/bench_summary.py gpurun_out/bench_${TAG}_off.json
