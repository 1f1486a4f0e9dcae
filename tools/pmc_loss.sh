# usage: bash tools/pmc_loss.sh TAG — loss-only pass (N=128, T=2e7): kernel trace + clock/issue PMC + LDS counters
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/pmc_loss_$TAG
mkdir -p $O
timeout -k 10 120 python3 tools/bench_loss.py 128 2e7 5 > $O/bench.txt 2>&1 || { cat $O/bench.txt; exit 1; }
cat $O/bench.txt
CLK="GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CLK -d $O/clock -o run --output-format csv -- python3 tools/bench_loss.py 128 2e7 3 auto > $O/clock.log 2>&1 || { tail -5 $O/clock.log; exit 1; }
W="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $W -d $O/wait -o run --output-format csv -- python3 tools/bench_loss.py 128 2e7 3 auto > $O/wait.log 2>&1 || { tail -5 $O/wait.log; exit 1; }
python3 tools/pmc_kernels.py $O/clock.json /dev/null $O/clock
python3 tools/pmc_kernels.py $O/wait.json /dev/null $O/wait
