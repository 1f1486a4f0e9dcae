# usage: bash tools/prof_round.sh TAG  — bench + kernel trace + FETCH/WRITE_SIZE for the default workload
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --to-tol 0 --cpu-baseline 0 > gpurun_out/prof_${TAG}_bench.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcf_$TAG -o run --output-format csv -- python bench.py --steps 2 --warmup 0 --to-tol 0 --cpu-baseline 0 > gpurun_out/pmcf_${TAG}_bench.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw_$TAG -o run --output-format csv -- python bench.py --steps 2 --warmup 0 --to-tol 0 --cpu-baseline 0 > gpurun_out/pmcw_${TAG}_bench.log 2>&1 || exit 1
cat gpurun_out/bench_$TAG.json
