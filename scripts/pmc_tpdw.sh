# PMC passes (one rocprofv3 run each) over the K7f microbenchmark; results under gpurun_out/pmc_tpdw
#   bash scripts/pmc_tpdw.sh [fused|unfused] [kernel-name substring]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_tpdw
i=0
for pmc in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL" \
           "FETCH_SIZE TCC_HIT_sum" "TCC_MISS_sum WRITE_SIZE" "SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/pmc_tpdw/p$i -o p -- python3 scripts/mb_tpdw.py ${1:-fused} > gpurun_out/pmc_tpdw/p$i.log 2>&1 || exit $?
done
KNAME=${2:-tp_node_dw} python3 - <<'PY'
import csv, glob, collections, os
for f in sorted(glob.glob("gpurun_out/pmc_tpdw/p*/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if os.environ["KNAME"] in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in acc.items():
        print(k, "per launch", sum(v) / len(v), "n", len(v))
PY
