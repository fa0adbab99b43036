# MSD + LDS bucket sort: GPU parity suite, survey of the workloads
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${T:-r3l}
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 150 --timeout-method thread > gpurun_out/${T}_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/${T}_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.txt
RUNS="mixed: sw_bursty: fw_uniform: tb_zipf: mixed:routed" bash scripts/survey.sh > gpurun_out/${T}_survey.txt 2>&1
cat gpurun_out/${T}_survey.txt
