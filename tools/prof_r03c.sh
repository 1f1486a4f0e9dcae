# usage: bash tools/prof_r03c.sh TAG — round-3 profile set under gpurun_out/prof_TAG/:
#   C3 (bench.py, 2 timed steps): clock/issue PMC + kernel trace, FETCH_SIZE, WRITE_SIZE passes;
#   C3 kernel trace --stats of the default bench command (no CPU baseline, no other configs);
#   C4 (tools/run_configs.py, 12 iterations): clock PMC + kernel trace, FETCH, WRITE; C4 --stats;
#   C5 kernel trace --stats and clock PMC LAST (rocprofv3 SIGSEGVs in exit() after writing its
#   output when the JADE device sweeps ran).
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/prof_$TAG
mkdir -p $O
CLK="GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY"
B3="python3 bench.py --steps 2 --warmup 0 --to-tol 0 --cpu-baseline 0 --configs 0"
pass() {  # pass NAME SECONDS ROCPROF-ARGS... -- CMD...
  local name=$1 secs=$2; shift 2
  echo "[prof] $name"
  timeout -s KILL $secs rocprofv3 "$@" > $O/$name.log 2>&1 || { echo "[prof] $name failed"; tail -30 $O/$name.log; exit 1; }
}
pass c3_clock 240 --kernel-trace --pmc $CLK -d $O/c3_clock -o run --output-format csv -- $B3
pass c3_fetch 240 --pmc FETCH_SIZE -d $O/c3_fetch -o run --output-format csv -- $B3
pass c3_write 240 --pmc WRITE_SIZE -d $O/c3_write -o run --output-format csv -- $B3
pass c3_trace 300 --kernel-trace --stats -d $O/c3_trace -o run --output-format csv -- python3 bench.py --cpu-baseline 0 --configs 0
R4="python3 tools/run_configs.py C4 --max-iter=12"
pass c4_clock 300 --kernel-trace --pmc $CLK -d $O/c4_clock -o run --output-format csv -- $R4
pass c4_fetch 300 --pmc FETCH_SIZE -d $O/c4_fetch -o run --output-format csv -- $R4
pass c4_write 300 --pmc WRITE_SIZE -d $O/c4_write -o run --output-format csv -- $R4
pass c4_trace 300 --kernel-trace --stats -d $O/c4_trace -o run --output-format csv -- python3 tools/run_configs.py C4
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/c5_trace -o run --output-format csv -- python3 tools/run_configs.py C5 > $O/c5_trace.log 2>&1
echo "[prof] c5_trace rc=$? (139 = the known SIGSEGV in exit() after the output was written)"
