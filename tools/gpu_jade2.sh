# usage: bash tools/gpu_jade2.sh TAG — JADE tests, C5 twice with the warm-start trace, then the kernel
# trace of C5
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_jade.py tests/test_gpu_parity.py -k "jade" -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_jade_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_jade_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_jade_$TAG.log
for i in 1 2; do
  PICARD_TRACE=1 timeout -k 10 200 python3 tools/run_configs.py C5 > gpurun_out/c5_$TAG.$i.json 2> gpurun_out/c5_$TAG.$i.log || exit 1
  echo "run $i: $(grep 'jade:' gpurun_out/c5_$TAG.$i.log)"
done
O=gpurun_out/prof_$TAG
mkdir -p $O
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/c5_trace -o run --output-format csv -- python3 tools/run_configs.py C5 > $O/c5_trace.log 2>&1
echo "c5_trace rc=$?"
grep -h "k_jade_sweeps\|k_moments4" $O/c5_trace/run_kernel_stats.csv | cut -d, -f2-4
