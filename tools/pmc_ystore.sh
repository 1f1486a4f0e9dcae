# usage: bash tools/pmc_ystore.sh TAG — k_ystore timing, clock/issue PMC pass, FETCH/WRITE passes
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/pmc_ys_$TAG
mkdir -p $O
timeout -k 10 120 python3 tools/bench_transform.py 128 2e7 5 > $O/bench.txt 2>&1 || { cat $O/bench.txt; exit 1; }
cat $O/bench.txt
timeout -k 10 120 python3 tools/bench_transform.py 128 1e8 3 >> $O/bench.txt 2>&1 || { cat $O/bench.txt; exit 1; }
tail -1 $O/bench.txt
CLK="GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CLK -d $O/clock -o run --output-format csv -- python3 tools/bench_transform.py 128 2e7 3 > $O/clock.log 2>&1 || { tail -5 $O/clock.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 tools/bench_transform.py 128 2e7 3 > $O/fetch.log 2>&1 || { tail -5 $O/fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 tools/bench_transform.py 128 2e7 3 > $O/write.log 2>&1 || { tail -5 $O/write.log; exit 1; }
echo done
