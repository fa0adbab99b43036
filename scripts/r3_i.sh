# routed path with the host-planned merge: route GPU tests + routed survey lines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${T:-r3i}
timeout -k 10 300 python -u -m pytest tests/test_route_gpu.py -m gpu -q -x --timeout 150 --timeout-method thread > gpurun_out/${T}_gpu_tests.txt 2>&1 || { tail -30 gpurun_out/${T}_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.txt
RUNS="mixed:routed tb_zipf:routed mixed:" bash scripts/survey.sh > gpurun_out/${T}_survey.txt 2>&1
cat gpurun_out/${T}_survey.txt
python - <<'PY'
import json
for n in ("mixed_routed", "tb_zipf_routed"):
    d = json.load(open(f"gpurun_out/survey/{n}.json"))
    print(n, d["config"].get("host_ms_per_step"))
PY
TAG=${T}_routed bash scripts/prof_routed.sh
