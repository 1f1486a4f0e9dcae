# usage: bash tools/prof_round.sh TAG — bench (with CPU baseline) + kernel trace + FETCH/WRITE_SIZE passes
# for the default workload; everything lands in gpurun_out/round_TAG/ (copy to profiles/TAG afterwards).
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/round_$TAG
mkdir -p $O
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmcf -o run --output-format csv -- python3 bench.py --steps 2 --warmup 0 --to-tol 0 --cpu-baseline 0 > $O/pmcf_bench.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmcw -o run --output-format csv -- python3 bench.py --steps 2 --warmup 0 --to-tol 0 --cpu-baseline 0 > $O/pmcw_bench.log 2>&1 || exit 1
python3 tools/pmc_summary.py 128 100000000 profiles/pmc_latest.json $O/pmcf/run_counter_collection.csv $O/pmcw/run_counter_collection.csv > $O/pmc_summary.json || exit 1
cp profiles/pmc_latest.json $O/pmc_latest.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --cpu-baseline 0 > $O/trace_bench.json 2> $O/trace_bench.err || exit 1
timeout -k 10 500 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 1
cat $O/bench.json
