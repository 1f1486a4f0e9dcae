# usage: bash tools/pmc_clock.sh TAG — effective clock (GRBM_GUI_ACTIVE / 8 / duration) and issue mix
# of the bench's kernels (one --pmc pass with --kernel-trace, same bench command as prof_round.sh)
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/clock_$TAG
mkdir -p $O
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY -d $O/p1 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 0 --to-tol 0 --cpu-baseline 0 ${BENCH_ARGS} > $O/p1.log 2>&1 || exit 1
python3 tools/clock_summary.py $O/p1 > $O/summary.txt || exit 1
cat $O/summary.txt
