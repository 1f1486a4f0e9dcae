# usage: bash tools/prof_c4.sh TAG — the C4 profile set under gpurun_out/prof_TAG/ (round 5):
#   C4 (tools/run_configs.py, 12 iterations): clock / issue PMC + kernel trace, FETCH_SIZE,
#   WRITE_SIZE (one pass each), then --kernel-trace --stats of the whole C4 fit; the table:
#   python3 tools/pmc_table.py gpurun_out/prof_TAG c4
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/prof_$TAG
mkdir -p $O
CLK="GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY"
pass() {  # pass NAME SECONDS ROCPROF-ARGS... -- CMD...
  local name=$1 secs=$2; shift 2
  echo "[prof] $name"
  timeout -s KILL $secs rocprofv3 "$@" > $O/$name.log 2>&1 || { echo "[prof] $name failed"; tail -30 $O/$name.log; exit 1; }
}
R4="python3 tools/run_configs.py C4 --max-iter=12"
pass c4_clock 300 --kernel-trace --pmc $CLK -d $O/c4_clock -o run --output-format csv -- $R4
pass c4_fetch 300 --pmc FETCH_SIZE -d $O/c4_fetch -o run --output-format csv -- $R4
pass c4_write 300 --pmc WRITE_SIZE -d $O/c4_write -o run --output-format csv -- $R4
pass c4_trace 300 --kernel-trace --stats -d $O/c4_trace -o run --output-format csv -- python3 tools/run_configs.py C4
python3 tools/pmc_table.py $O c4 > $O/c4_pmc_table.txt && cat $O/c4_pmc_table.txt
