# usage: bash tools/prof_final.sh TAG — HEAD profile set: bench under --kernel-trace --stats (one
# process), then FETCH_SIZE / WRITE_SIZE / clock passes over 4 timed bench steps (each pass time-limited)
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/proff_$TAG
mkdir -p $O
B="python3 bench.py --cpu-baseline 0 --configs 0 --to-tol 0"
timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
  python3 bench.py --cpu-baseline 0 --configs 0 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 tools/bench_summary.py $O/bench.json
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- $B --steps 4 --warmup 5 > $O/fetch.log 2>&1 || { tail -5 $O/fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- $B --steps 4 --warmup 5 > $O/write.log 2>&1 || { tail -5 $O/write.log; exit 1; }
CLK="GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS"
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $CLK -d $O/clock -o run --output-format csv -- $B --steps 4 --warmup 5 > $O/clock.log 2>&1 || { tail -5 $O/clock.log; exit 1; }
echo done
