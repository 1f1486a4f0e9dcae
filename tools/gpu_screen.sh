# usage: bash tools/gpu_screen.sh TAG — screen / int8 GPU tests, screen timing, C3 bench (no other configs)
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_screen32.py tests/test_gpu_int8.py tests/test_gpu_group.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_screen_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_screen_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_screen_$TAG.log
timeout -k 10 120 python3 tools/bench_loss.py 128 2e7 5 auto || exit 1
timeout -k 10 120 python3 tools/bench_loss.py 64 1e6 20 auto || exit 1
timeout -k 10 400 python bench.py --cpu-baseline 0 --configs 0 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
python3 tools/bench_summary.py gpurun_out/bench_$TAG.json
PICARD_TRACE=1 timeout -k 10 120 python3 tools/run_configs.py C2 > gpurun_out/c2_$TAG.json 2> gpurun_out/c2_trace_$TAG.txt || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/c2_$TAG.json')); print({k: d[k] for k in ('iterations_s','n_iterations','samples_per_s_per_iter','passes')})"
