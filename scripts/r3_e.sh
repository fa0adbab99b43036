# dual grouping streams (A/B RL_FRONTS=1/2) and zero-copy coalescer batches (A/B)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 150 --timeout-method thread > gpurun_out/r3e_gpu_tests.txt 2>&1 || { tail -30 gpurun_out/r3e_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r3e_gpu_tests.txt
for f in 2 1 2 1; do
  echo "RL_FRONTS=$f"
  RL_FRONTS=$f RUNS="tb_zipf: mixed: sw_bursty: fw_uniform:" bash scripts/survey.sh || exit $?
done > gpurun_out/r3e_fronts.txt 2>&1
cat gpurun_out/r3e_fronts.txt
for zc in 65536 0; do
  RL_COALESCER_ZC_MAX=$zc timeout -k 10 200 python bench.py --e2e --qps 1e5,1e6,3e6 --seconds 8 > gpurun_out/r3e_e2e_zc$zc.json 2> gpurun_out/r3e_e2e_zc$zc.err || { tail gpurun_out/r3e_e2e_zc$zc.err; exit 1; }
  python - gpurun_out/r3e_e2e_zc$zc.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for l in d["levels"]:
    print(sys.argv[1], l["offered_qps"], "p50", l["p50_us"], "p99", l["p99_us"], "p999", l["p999_us"], "max100ms", max(l["max_us_by_100ms"]))
PY
done
