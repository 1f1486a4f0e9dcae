# usage: bash tools/pmc_oz.sh TAG — loss + fused passes (N=128, T=2e7) on both Y stages:
# timings, then clock/issue PMC and FETCH/WRITE passes of the int8 kernels (each pass time-limited)
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/pmc_oz_$TAG
mkdir -p $O
timeout -k 10 120 python3 tools/bench_loss.py 128 2e7 5 > $O/bench.txt 2>&1 || { cat $O/bench.txt; exit 1; }
cat $O/bench.txt
CLK="GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS"
for m in auto f64; do
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CLK -d $O/clock_$m -o run --output-format csv -- python3 tools/bench_loss.py 128 2e7 3 $m > $O/clock_$m.log 2>&1 || { tail -5 $O/clock_$m.log; exit 1; }
done
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 tools/bench_loss.py 128 2e7 3 auto > $O/fetch.log 2>&1 || { tail -5 $O/fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 tools/bench_loss.py 128 2e7 3 auto > $O/write.log 2>&1 || { tail -5 $O/write.log; exit 1; }
echo done
