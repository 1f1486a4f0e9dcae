# usage: bash tools/gpu_screen_clock.sh TAG — the screen's and the fused pass's clock (GRBM_GUI_ACTIVE
# over kernel time) at T = 4e5 (the screen's 4 digit planes, 205 MB, fit the 256 MB Infinity Cache),
# 2e6 and 2e7 (HBM-streamed): is the screen's low clock the memory side's power?
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/sclk_$TAG
mkdir -p $O
for t in 4e5 2e6 2e7; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --kernel-include-regex "screen|fused" --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA \
    -d $O/t$t/p1 -o run --output-format csv -- python3 tools/bench_loss.py 128 $t 20 auto > $O/t$t.log 2>&1 || { tail -5 $O/t$t.log; exit 1; }
  echo "== T=$t"; grep -E "screen|fused" $O/t$t.log
  python3 tools/screen_pmc.py $O/t$t | grep -E "launches|MFMA_BUSY"
done
