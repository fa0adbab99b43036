#!/bin/bash
# SQ counters of k_tb_chain on the single-hot-key workload (one block does all
# the work, so the counters describe the chain/producer/loader waves).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
B="python3 bench.py --workload ${WL:-tb_hot} --steps 3 --warmup 1 --no-cpu-baseline"
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc/p$i -o run -- $B > gpurun_out/pmc/p$i.log 2>&1 || exit $?
done
python3 - <<'PY'
import csv, collections, glob
for f in sorted(glob.glob("gpurun_out/pmc/p*/run_counter_collection.csv")):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "k_tb_chain" in r["Kernel_Name"]:
            d[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f, {k: v[-1] for k, v in d.items()})
PY
