# usage: bash tools/prof_r03b.sh TAG — C2 / C5 line-search traces (host vs device time per
# iteration), C2 kernel trace, then the C5 clock PMC pass LAST (rocprofv3 SIGSEGVs in exit()
# after writing its output when the JADE device sweeps ran: DESIGN.md §6).
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/prof_$TAG
mkdir -p $O
PICARD_TRACE=1 timeout -k 10 120 python3 tools/run_configs.py C2 > $O/c2_run.json 2> $O/c2_trace.err || exit 1
PICARD_TRACE=1 timeout -k 10 120 python3 tools/run_configs.py C5 > $O/c5_run.json 2> $O/c5_trace.err || exit 1
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/c2_ktrace -o run --output-format csv -- python3 tools/run_configs.py C2 > $O/c2_ktrace.log 2>&1 || exit 1
CLK="GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY"
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $CLK -d $O/c5_clock -o run --output-format csv -- python3 tools/run_configs.py C5 --max-iter=3 > $O/c5_clock.log 2>&1
echo "c5_clock rc=$?"
