# probe A/B on mixed: rows per thread (PROBE_R) x grid
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for cfg in "1 1024" "2 1024" "4 1024" "1 4096" "2 2048" "1 1024"; do
  set -- $cfg
  RL_PROBE_R=$1 RL_PROBE_GRID=$2 RUNS="mixed: sw_bursty:" bash scripts/survey.sh | sed "s/^/R=$1 grid=$2 /"
done
