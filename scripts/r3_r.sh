# round-3 checkpoint: GPU suite, smoke, bench, rocprofv3 (configs[1], mixed) with PMC, survey, gRPC and e2e levels
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${T:-r3r}
T=$T bash scripts/r3_f.sh || exit $?
timeout -k 10 400 python bench.py --grpc --seconds 3 --grpc-unary 10000,35000,70000,100000,150000 > gpurun_out/${T}_grpc.json 2> gpurun_out/${T}_grpc.err || { tail -20 gpurun_out/${T}_grpc.err; exit 1; }
grep '^{' gpurun_out/${T}_grpc.err || true
timeout -k 10 300 python bench.py --e2e --qps 1e5,1e6,3e6,1e7 --seconds 4 > gpurun_out/${T}_e2e.json 2> gpurun_out/${T}_e2e.err || { tail -20 gpurun_out/${T}_e2e.err; exit 1; }
python - gpurun_out/${T}_e2e.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for l in d["levels"]:
    print("e2e", l["offered_qps"], "p50", l["p50_us"], "p99", l["p99_us"], "p999", l["p999_us"], "mean batch", l.get("mean_batch"))
PY
