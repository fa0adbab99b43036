"""bench.py's N > 1 path, rehearsed on one GPU (GPU).

The driver runs `bench.py --gpus N` on an 8-GPU node this pipeline never
gives us; this runs the same code path -- torch.distributed.run with two
ranks, the routed Zipf headline, the hot-owner bound, the configs[3]
secondaries under their own metric names -- with both ranks on GPU 0 and the
collectives over gloo (--rehearse-gloo).  It checks the line's shape, not its
numbers (two ranks share one GPU)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_rehearsal():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--rehearse-gloo", "--steps", "3",
           "--warmup", "1", "--batch", "200000", "--lat-batches", "0", "--no-cpu-baseline"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=240, env=env)
    lines = [ln for ln in p.stdout.decode().splitlines() if ln.startswith("{")]
    assert p.returncode == 0 and lines, p.stderr.decode()[-3000:]
    d = json.loads(lines[-1])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["steps"] == 3
    # the headline is BASELINE's own metric on its own workload (Zipf 1M keys), routed
    assert d["metric"].startswith("decisions/sec @1/8 GPU, Zipf 1M keys")
    assert d["config"]["workload"].startswith("configs[1]")
    assert d["config"]["parallelism"].startswith("routed")
    assert d["value"] > 0 and d["roofline"]["frac"] > 0
    hob = d["hot_owner_bound"]
    assert hob and hob["hot_share"] > 0.05 and hob["bound_decisions_per_s"] > 0
    # configs[3] beside it, routed and as replicas, each under its own metric name
    sec = d["secondary"]
    assert len(sec) == 2 and all("error" not in s for s in sec), sec
    assert all(s["metric"].startswith("decisions/sec @2 GPU, configs[3]") for s in sec)
    assert {s["ingress"].split(":")[0].split(" ")[0] for s in sec} == {"routed", "sharded"}
