cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS -d gpurun_out/pmc_split1 -o run --output-format csv -- python tools/bench_split.py 128 2e7 2 > gpurun_out/pmc_split1.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU -d gpurun_out/pmc_split2 -o run --output-format csv -- python tools/bench_split.py 128 2e7 2 > gpurun_out/pmc_split2.log 2>&1 || exit 1
python3 - <<'PY'
import csv, collections
for f in ["gpurun_out/pmc_split1/run_counter_collection.csv","gpurun_out/pmc_split2/run_counter_collection.csv"]:
    agg=collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        k=r["Kernel_Name"]
        if "k_eval" not in k: continue
        agg[k.split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k,v in agg.items():
        print(k, {c: sum(x)/len(x) for c,x in v.items()})
PY
