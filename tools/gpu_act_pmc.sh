# SQ counters of the act kernel (one pass, 8 SQ counters)
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/actpmc
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/actpmc -o pmc -- python tools/act_bench.py > gpurun_out/actpmc/out.txt 2>&1 || exit 1
f=$(find gpurun_out/actpmc -name "*counter_collection.csv" | head -1)
python - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if "sc_act" in r.get("Kernel_Name", ""):
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(k, "mean per dispatch %.4g" % (sum(v) / len(v)), "n", len(v))
PY
