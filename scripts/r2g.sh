cd "${GRAFT_REPO_ROOT}"
STEPS=tests bash scripts/gpu_check.sh || exit $?
grep -q " passed" gpurun_out/gpu_tests.log && ! grep -q "failed" gpurun_out/gpu_tests.log || { echo TESTS-FAILED; exit 1; }
BARGS="--lat-batches 0" STEPS=12 bash scripts/ab.sh librl_amd_base.so librl_amd.so > gpurun_out/ab_tables.txt 2>&1 || exit $?
BARGS="--workload tb_zipf15 --lat-batches 0" STEPS=8 bash scripts/ab.sh librl_amd_base.so librl_amd.so >> gpurun_out/ab_tables.txt 2>&1 || exit $?
RL_AMD_LIB=$PWD/distributed-rate-limiter_amd/lib/librl_amd_stamps.so TAG=stamps_tables bash scripts/bench_brief.sh > gpurun_out/stamps_tables.txt 2>&1
