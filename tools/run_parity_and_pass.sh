timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1; tail -3 gpurun_out/gpu_tests.log
for n in 128 64 32 16; do timeout -k 10 100 python tools/bench_pass.py $n 2e7 tanh 5 || exit 1; done
timeout -k 10 100 python tools/bench_pass.py 128 2e7 exp 5 && timeout -k 10 100 python tools/bench_pass.py 128 2e7 cube 5 && timeout -k 10 100 python tools/bench_pass.py 64 2e7 tanh 5 1
