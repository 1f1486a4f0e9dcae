# usage: bash tools/gpu_c4.sh TAG [pytest-args] — GPU parity tests (time-limited), then a C4 kernel
# trace (12 iterations) and a C3 bench (no CPU baseline), all under gpurun_out/
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/c4_$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest ${@:-tests} -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
  python3 tools/run_configs.py C4 --max-iter=12 > $O/c4.log 2>&1 || { tail -20 $O/c4.log; exit 1; }
python3 -c "
import csv,glob
f=glob.glob('$O/trace/**/run_kernel_stats.csv',recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:10]: print('%-60s n=%5s avg %.3f ms tot %.1f ms'%(r['Name'][:60],r['Calls'],float(r['AverageNs'])/1e6,float(r['TotalDurationNs'])/1e6))"
timeout -k 10 400 python bench.py --cpu-baseline 0 --steps 10 --warmup 2 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 tools/bench_summary.py $O/bench.json
