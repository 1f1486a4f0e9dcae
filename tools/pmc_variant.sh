# usage: bash tools/pmc_variant.sh v1 v2 ... — clock + issue-mix PMC (two passes) of bench_split (N=128, T=5e7)
# for each variants/<v>.so
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PICARD_NO_YSTORE=1
cp picard-ica_amd/libpicard_mi355x.so /tmp/orig.so
for v in "$@"; do
  cp variants/$v.so picard-ica_amd/libpicard_mi355x.so
  O=gpurun_out/pmcv_$v; mkdir -p $O
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY -d $O/p1 -o run --output-format csv -- python3 tools/bench_split.py 128 5e7 2 tanh 0.3 > $O/p1.log 2>&1 || { cp /tmp/orig.so picard-ica_amd/libpicard_mi355x.so; exit 1; }
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM -d $O/p2 -o run --output-format csv -- python3 tools/bench_split.py 128 5e7 2 tanh 0.3 > $O/p2.log 2>&1 || { cp /tmp/orig.so picard-ica_amd/libpicard_mi355x.so; exit 1; }
  echo "== $v"; python3 tools/clock_summary.py $O/p1; python3 tools/clock_summary.py $O/p2
done
cp /tmp/orig.so picard-ica_amd/libpicard_mi355x.so
