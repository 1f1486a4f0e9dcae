# usage: bash tools/gpu_g8.sh TAG — the digit-G tests, pass timings with and without the digit G
# stage at (128, 2e7), then the driver-window bench
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
# (a failing assertion does not stop the timings below; a crash or time-out does)
timeout -k 10 600 python -u -m pytest tests/test_gpu_g8.py tests/test_gpu_int8.py tests/test_gpu_parity.py -m gpu -q \
  --timeout 300 --timeout-method thread > gpurun_out/g8tests_$TAG.log 2>&1; rc=$?
tail -4 gpurun_out/g8tests_$TAG.log
[ $rc -le 1 ] || exit 1
timeout -k 10 120 python -u tools/bench_pass.py 128 2e7 tanh 5 > gpurun_out/pass_$TAG.txt 2>&1 || { tail -20 gpurun_out/pass_$TAG.txt; exit 1; }
PICARD_G8=0 timeout -k 10 120 python -u tools/bench_pass.py 128 2e7 tanh 5 >> gpurun_out/pass_$TAG.txt 2>&1 || { tail -20 gpurun_out/pass_$TAG.txt; exit 1; }
cat gpurun_out/pass_$TAG.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_golden.py tests/test_gpu_fullsize_fit.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/fit_$TAG.log 2>&1 || { tail -60 gpurun_out/fit_$TAG.log; exit 1; }
tail -2 gpurun_out/fit_$TAG.log
timeout -k 10 600 python -u bench.py --warmup 5 --steps 20 --configs 0 --cpu-baseline 0 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
python3 tools/bench_summary.py gpurun_out/bench_$TAG.json
