# usage: bash tools/gpu_oz.sh TAG — int8-slice Y stage: its GPU tests, loss-pass timing + clock PMC, bench
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_int8.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_oz_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_oz_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_oz_$TAG.log
timeout -k 10 120 python3 tools/bench_loss.py 128 2e7 5 || exit 1
O=gpurun_out/pmc_loss_$TAG
CLK="GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CLK -d $O -o run --output-format csv -- python3 tools/bench_loss.py 128 2e7 3 auto > $O.log 2>&1 || { tail -5 $O.log; exit 1; }
timeout -k 10 400 python bench.py --cpu-baseline 0 --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
python3 tools/bench_summary.py gpurun_out/bench_$TAG.json
