#!/bin/bash
# Round checkpoint on a GPU box: GPU suite, smoke, bench, rocprofv3 kernel
# stats + FETCH/WRITE passes (configs[1] as the bench runs it, mixed), per-workload survey,
# then (FULL=1) the gRPC levels and the coalescer e2e levels.
# Usage: T=<tag> [FULL=1] bash scripts/checkpoint.sh   (outputs: gpurun_out/<tag>_*)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${T:-ckpt}
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 150 --timeout-method thread > gpurun_out/${T}_gpu_tests.txt 2>&1 || { tail -30 gpurun_out/${T}_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1 || { tail -20 gpurun_out/${T}_smoke.txt; exit 1; }
cat gpurun_out/${T}_smoke.txt
timeout -k 10 300 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
cat gpurun_out/${T}_bench.json
TAG=${T}_zipf BARGS="--no-cpu-baseline" bash scripts/profile.sh > gpurun_out/${T}_prof_zipf.txt 2>&1 || { cat gpurun_out/${T}_prof_zipf.txt; exit 1; }
TAG=${T}_mixed BARGS="--workload mixed --steps 10 --warmup 2 --no-cpu-baseline --lat-batches 0" bash scripts/profile.sh > gpurun_out/${T}_prof_mixed.txt 2>&1 || { cat gpurun_out/${T}_prof_mixed.txt; exit 1; }
bash scripts/survey.sh > gpurun_out/${T}_survey.txt 2>&1
cat gpurun_out/${T}_survey.txt
[ -n "$FULL" ] || exit 0
timeout -k 10 400 python bench.py --grpc --seconds 3 --grpc-unary 10000,35000,70000,100000,150000 > gpurun_out/${T}_grpc.json 2> gpurun_out/${T}_grpc.err || { tail -20 gpurun_out/${T}_grpc.err; exit 1; }
grep '^{' gpurun_out/${T}_grpc.err || true
timeout -k 10 300 python bench.py --e2e --qps 1e5,1e6,3e6,1e7 --seconds 4 > gpurun_out/${T}_e2e.json 2> gpurun_out/${T}_e2e.err || { tail -20 gpurun_out/${T}_e2e.err; exit 1; }
python - gpurun_out/${T}_e2e.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for l in d["levels"]:
    print("e2e", l["offered_qps"], "p50", l["p50_us"], "p99", l["p99_us"], "p999", l["p999_us"], "mean batch", l.get("mean_batch"))
PY
