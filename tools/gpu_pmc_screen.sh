# usage: bash tools/gpu_pmc_screen.sh TAG — stall breakdown of the screen (bench_loss 128 2e7, screen only)
# and the C5 FETCH / WRITE passes (JADE moments traffic; these exit with the known rocprofv3 crash)
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/pmcs_$TAG
mkdir -p $O
W="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $W -d $O/screen_wait -o run --output-format csv -- python3 tools/bench_loss.py 128 2e7 3 auto > $O/screen_wait.log 2>&1 || { tail -20 $O/screen_wait.log; exit 1; }
V="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $V -d $O/screen_inst -o run --output-format csv -- python3 tools/bench_loss.py 128 2e7 3 auto > $O/screen_inst.log 2>&1 || { tail -20 $O/screen_inst.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/c5_fetch -o run --output-format csv -- python3 tools/run_configs.py C5 > $O/c5_fetch.log 2>&1
echo "c5 fetch rc=$?"
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/c5_write -o run --output-format csv -- python3 tools/run_configs.py C5 > $O/c5_write.log 2>&1
echo "c5 write rc=$?"
exit 0
