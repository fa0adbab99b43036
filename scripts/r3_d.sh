# configs[4] stall attribution under a HIP API trace, then the hot-key workloads
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf /tmp/stall
RL_COALESCER_TRACE=65536 timeout -s KILL 180 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d /tmp/stall -o run -- distributed-rate-limiter_amd/lib/rl_bench_e2e --qps 3e6 --seconds 4 > gpurun_out/r3d_stall_e2e.json 2> gpurun_out/r3d_stall_e2e.err || { tail gpurun_out/r3d_stall_e2e.err; exit 1; }
python scripts/stall_trace.py /tmp/stall gpurun_out/r3d_stall_trace.json || exit 1
RUNS="tb_zipf15: tb_hot: mixed:routed" bash scripts/survey.sh > gpurun_out/r3d_survey.txt 2>&1 || exit $?
cat gpurun_out/r3d_survey.txt
