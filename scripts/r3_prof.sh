set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/survey.sh > gpurun_out/r3a_survey.txt 2>&1 || exit $?
TAG=r3a_mixed BARGS="--workload mixed --steps 10 --warmup 2 --no-cpu-baseline --lat-batches 0" bash scripts/profile.sh > gpurun_out/r3a_prof_mixed.txt 2>&1 || exit $?
TAG=r3a_zipf BARGS="--steps 10 --warmup 2 --no-cpu-baseline --lat-batches 0" bash scripts/profile.sh > gpurun_out/r3a_prof_zipf.txt 2>&1
