# round 3 GPU batch: parity suite, survey of the main workloads, e2e without
# tracing, then the configs[4] stall attribution under a HIP API trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 150 --timeout-method thread > gpurun_out/r3b_gpu_tests.txt 2>&1 || { tail -30 gpurun_out/r3b_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r3b_gpu_tests.txt
RUNS="tb_zipf: mixed: sw_bursty: fw_uniform:" bash scripts/survey.sh > gpurun_out/r3b_survey.txt 2>&1 || exit $?
cat gpurun_out/r3b_survey.txt
timeout -k 10 120 python bench.py --e2e --qps 1e5,1e6,3e6 --seconds 2 > gpurun_out/r3b_e2e.json 2> gpurun_out/r3b_e2e.err || { tail gpurun_out/r3b_e2e.err; exit 1; }
rm -rf /tmp/stall
RL_COALESCER_TRACE=65536 timeout -s KILL 180 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d /tmp/stall -o run -- distributed-rate-limiter_amd/lib/rl_bench_e2e --qps 3e6 --seconds 3 > gpurun_out/r3b_stall_e2e.json 2> gpurun_out/r3b_stall_e2e.err || { tail gpurun_out/r3b_stall_e2e.err; exit 1; }
python scripts/stall_trace.py /tmp/stall gpurun_out/r3b_stall_trace.json
