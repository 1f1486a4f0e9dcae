# usage: bash tools/prof_c4.sh — kernel trace of the C4 config (N=256 non-ortho) end to end
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/prof_c4; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv -- python3 tools/run_configs.py C4 > $O/c4.json 2> $O/c4.err || exit 1
head -12 $O/run_kernel_stats.csv | cut -c1-250
