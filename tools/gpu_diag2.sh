# usage: bash tools/gpu_diag2.sh TAG — C5 kernel trace with pc_device_release before exit (the
# rocprofv3 exit crash), then the C2 HIP-API trace (per-call host cost of the solver's passes)
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/diag_$TAG
mkdir -p $O
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/c5_trace -o run --output-format csv -- python3 tools/run_configs.py C5 --release > $O/c5_trace.log 2>&1
echo "c5 trace (with --release) rc=$?"
tail -5 $O/c5_trace.log
timeout -s KILL 200 rocprofv3 --runtime-trace --stats -d $O/c2_api -o run --output-format csv -- python3 tools/run_configs.py C2 --release > $O/c2_api.log 2>&1
echo "c2 api rc=$?"
ls $O/c2_api
exit 0
