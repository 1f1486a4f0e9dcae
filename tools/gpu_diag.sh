# usage: bash tools/gpu_diag.sh TAG — C2 per-iteration trace (PICARD_TRACE) and the C5 rocprofv3
# exit crash with /proc/self/maps dumped at interpreter exit (tools/run_configs.py --maps)
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/diag_$TAG
mkdir -p $O
PICARD_TRACE=1 timeout -k 10 120 python3 tools/run_configs.py C2 > $O/c2.json 2> $O/c2_trace.txt || { tail -20 $O/c2_trace.txt; exit 1; }
python3 -c "import json; d=json.load(open('$O/c2.json')); print({k: d[k] for k in ('setup_s','iterations_s','n_iterations','samples_per_s_per_iter','passes','kernels')})"
grep "picard-trace" $O/c2_trace.txt | head -12
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/c5_trace -o run --output-format csv -- python3 tools/run_configs.py C5 --maps=$O/maps_c5.txt > $O/c5_trace.log 2>&1
echo "c5 trace rc=$?"
tail -30 $O/c5_trace.log
exit 0
