# probe A/B: read-then-CAS vs CAS-first
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 150 --timeout-method thread -k "random or config0 or config3 or skewed or gc" > gpurun_out/r3v_tests.txt 2>&1 || { tail -30 gpurun_out/r3v_tests.txt; exit 1; }
RL_PROBE_CAS=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 150 --timeout-method thread -k "random or config0 or config3 or skewed or gc" >> gpurun_out/r3v_tests.txt 2>&1 || { tail -30 gpurun_out/r3v_tests.txt; exit 1; }
grep passed gpurun_out/r3v_tests.txt
for c in 0 1 0 1; do
  if [ $c = 1 ]; then export RL_PROBE_CAS=1; else unset RL_PROBE_CAS; fi
  RUNS="mixed: sw_bursty: fw_uniform: tb_zipf:" STEPS=20 bash scripts/survey.sh | sed "s/^/cas=$c /"
done
