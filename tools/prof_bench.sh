# usage: bash tools/prof_bench.sh TAG — the bench command itself under rocprofv3 --kernel-trace --stats
# (bench JSON and kernel trace from ONE process), then the C5 kernel trace (JADE kernels)
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/profb_$TAG
mkdir -p $O
timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d $O/c3 -o run --output-format csv -- \
  python3 bench.py --cpu-baseline 0 --configs 0 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 tools/bench_summary.py $O/bench.json
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/c5 -o run --output-format csv -- python3 tools/run_configs.py C5 > $O/c5.log 2>&1 || { tail -5 $O/c5.log; exit 1; }
tail -3 $O/c5.log
