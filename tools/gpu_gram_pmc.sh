# usage: bash tools/gpu_gram_pmc.sh — issue / stall counters of the tiled phase 2 (k_tiled_gram2) at (256, 5e6):
# three PMC passes of tools/bench_tiled.py → screen_pmc.py summary in gpurun_out/gpmc/summary.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/gpmc
mkdir -p $O
P1="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC"
P2="GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INST_CYCLES_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_THREAD_CYCLES_VALU"
P3="GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --kernel-include-regex gram2 --pmc $P -d $O/p$i -o run \
    --output-format csv -- python3 tools/bench_tiled.py 256 5e6 2 > $O/p$i.log 2>&1 || { tail -20 $O/p$i.log; exit 1; }
done
python3 tools/screen_pmc.py $O > $O/summary.txt && cat $O/summary.txt
