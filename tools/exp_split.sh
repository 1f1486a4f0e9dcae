PICARD_TRACE=1 timeout -k 10 400 python bench.py --cpu-baseline 0 > gpurun_out/bench_trace.json 2> gpurun_out/bench_trace.err
timeout -k 10 100 python tools/bench_split.py 128 2e7 5 && PICARD_NO_YSTORE=1 timeout -k 10 100 python tools/bench_split.py 128 2e7 5 && timeout -k 10 100 python tools/bench_split.py 64 2e7 5
timeout -k 10 300 python tools/bench_pass.py 256 1e7 tanh 2 1
