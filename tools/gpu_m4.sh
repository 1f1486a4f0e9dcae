# usage: bash tools/gpu_m4.sh TAG — JADE moments pass: its GPU tests, a C5 run, then
# rocprofv3 kernel trace and FETCH / WRITE passes on C5 (each pass exits with the known
# SIGSEGV in exit() after writing its output, DESIGN.md §6, so their status is not checked)
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/m4_$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "moments4 or jade or shard_moments or group" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
PICARD_TRACE=1 timeout -k 10 200 python -u tools/run_configs.py C5 > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
grep "jade" $O/c5.err; python3 -c "import json; d=json.load(open('$O/c5.json')); print({k: d[k] for k in ('setup_s','iterations_s','n_iterations','samples_per_s_per_iter','amari')})"
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 tools/run_configs.py C5 > $O/trace.log 2>&1
echo "trace rc=$?"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 tools/run_configs.py C5 > $O/fetch.log 2>&1
echo "fetch rc=$?"
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 tools/run_configs.py C5 > $O/write.log 2>&1
echo "write rc=$?"
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS -d $O/lds -o run --output-format csv -- python3 tools/run_configs.py C5 > $O/lds.log 2>&1
echo "lds rc=$?"
exit 0
