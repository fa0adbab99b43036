# round-3 checkpoint at HEAD: GPU suite, smoke, bench, rocprofv3 stats + FETCH/WRITE passes (configs[1], mixed)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${T:-r3f}
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 150 --timeout-method thread > gpurun_out/${T}_gpu_tests.txt 2>&1 || { tail -30 gpurun_out/${T}_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1 || { tail -20 gpurun_out/${T}_smoke.txt; exit 1; }
cat gpurun_out/${T}_smoke.txt
timeout -k 10 300 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
cat gpurun_out/${T}_bench.json
TAG=${T}_zipf BARGS="--steps 10 --warmup 2 --no-cpu-baseline --lat-batches 0" bash scripts/profile.sh > gpurun_out/${T}_prof_zipf.txt 2>&1 || { cat gpurun_out/${T}_prof_zipf.txt; exit 1; }
TAG=${T}_mixed BARGS="--workload mixed --steps 10 --warmup 2 --no-cpu-baseline --lat-batches 0" bash scripts/profile.sh > gpurun_out/${T}_prof_mixed.txt 2>&1 || { cat gpurun_out/${T}_prof_mixed.txt; exit 1; }
bash scripts/survey.sh > gpurun_out/${T}_survey.txt 2>&1
cat gpurun_out/${T}_survey.txt
