# chain near fixed point with 3-offset evaluations: chain parity tests, then the TB workloads
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${T:-r3q}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 150 --timeout-method thread -k "chain or zipf or hot or config1 or random or skewed" > gpurun_out/${T}_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/${T}_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.txt
RUNS="tb_zipf: tb_zipf15: tb_hot: tb_zipf:" bash scripts/survey.sh > gpurun_out/${T}_survey.txt 2>&1
cat gpurun_out/${T}_survey.txt
