#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over scripts/one_gemm256.py
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
rm -rf gpurun_out/pmc/*
i=0
for ctrs in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_SALU" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
            "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs -d gpurun_out/pmc/p$i -o run --output-format csv -- python scripts/one_gemm256.py > gpurun_out/pmc/log$i.txt 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc/log$i.txt; exit 1; }
done
for f in $(find gpurun_out/pmc -name "*counter_collection.csv" | sort); do
  echo "== $f"; python - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    k = r.get("Kernel_Name", "")
    if "g256" in k:
        agg[k[:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for kn, d in agg.items():
    print(kn)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {sum(v)/len(v):.4g}")
PY
done
