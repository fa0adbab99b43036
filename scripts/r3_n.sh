# k_sort_local v2: GPU parity suite, survey, mixed kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${T:-r3n}
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 150 --timeout-method thread > gpurun_out/${T}_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/${T}_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.txt
RUNS="mixed: sw_bursty: fw_uniform: tb_zipf:" bash scripts/survey.sh > gpurun_out/${T}_survey.txt 2>&1
cat gpurun_out/${T}_survey.txt
TAG=${T}_mixed NO_PMC=1 BARGS="--workload mixed --steps 10 --warmup 2 --no-cpu-baseline --lat-batches 0" bash scripts/profile.sh > /dev/null 2>&1 || exit 1
python - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/prof/r3n_mixed_trace/run_kernel_stats.csv')))
for r in rows[:16]:
    n=r['Name'].replace('(anonymous namespace)::','').split('(')[0].replace('void ','').replace('rl::','')
    print(f"{n[:40]:40s} {r['Calls']:>6} {float(r['AverageNs'])/1e3:9.1f}")
PY
