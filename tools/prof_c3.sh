# usage: bash tools/prof_c3.sh TAG — the C3 profile set under gpurun_out/prof_TAG/:
#   kernel trace --stats of the default C3 bench command (single and paired screens listed as
#   their own instantiations), then FETCH_SIZE and WRITE_SIZE passes (separate runs) over 6
#   timed steps, whose searches include paired screens.
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/prof_$TAG
mkdir -p $O
B3="python3 bench.py --steps 6 --warmup 0 --to-tol 0 --cpu-baseline 0 --configs 0"
pass() {  # pass NAME SECONDS ROCPROF-ARGS... -- CMD...
  local name=$1 secs=$2; shift 2
  echo "[prof] $name"
  timeout -s KILL $secs rocprofv3 "$@" > $O/$name.log 2>&1 || { echo "[prof] $name failed"; tail -30 $O/$name.log; exit 1; }
}
pass c3_trace 300 --kernel-trace --stats -d $O/c3_trace -o run --output-format csv -- python3 bench.py --cpu-baseline 0 --configs 0
pass c3_fetch 240 --pmc FETCH_SIZE -d $O/c3_fetch -o run --output-format csv -- $B3
pass c3_write 240 --pmc WRITE_SIZE -d $O/c3_write -o run --output-format csv -- $B3
