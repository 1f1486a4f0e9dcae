# usage: bash tools/prof_r03.sh TAG — round-3 profile set under gpurun_out/prof_TAG/:
#   C3 (bench.py, 2 timed steps): clock/issue PMC pass (+kernel trace), FETCH_SIZE, WRITE_SIZE;
#   C5 kernel trace with the host JADE sweeps, then with the device sweeps (the round-2 exit
#   SIGSEGV under rocprofv3; /proc/self/maps dumped at interpreter exit for addr2line).
# Each pass runs under its own time limit; the first failure ends the script.
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
R5="python3 tools/run_configs.py C5 --max-iter=3"
PICARD_HOST_JADE=1 pass c5_hostjade 300 --kernel-trace --stats -d $O/c5_hostjade -o run --output-format csv -- $R5 --maps=$O/c5_hostjade_maps.txt
pass c5_trace 300 --kernel-trace --stats -d $O/c5_trace -o run --output-format csv -- $R5 --maps=$O/c5_trace_maps.txt
echo "[prof] done"
