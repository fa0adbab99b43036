"""The reference's integration tests (internal/ratelimiter/*_integration_test.go),
replayed on a deterministic clock against
  * the CPU oracle + Go-layer glue (CPU; pins the oracle to the reference's own
    assertions), and
  * the product: C++ host mirror over the HIP engine (GPU).
Profile = miniredis, which is what the reference tests ran on.
"""
import pytest

import backends
import scenarios

IDS = [n for n, _ in scenarios.ALL]


@pytest.mark.parametrize("name,fn", scenarios.ALL, ids=IDS)
def test_scenario_oracle(name, fn):
    fn(backends.OracleBackend(profile=1))


@pytest.mark.parametrize("name,fn", scenarios.ALL, ids=IDS)
def test_scenario_oracle_redis7(name, fn):
    # the canonical profile must satisfy the same assertions
    fn(backends.OracleBackend(profile=0))


@pytest.mark.gpu
@pytest.mark.parametrize("name,fn", scenarios.ALL, ids=IDS)
def test_scenario_gpu(name, fn):
    fn(backends.GpuBackend(profile=1))


@pytest.mark.gpu
@pytest.mark.parametrize("name,fn", scenarios.ALL, ids=IDS)
def test_scenario_gpu_redis7(name, fn):
    fn(backends.GpuBackend(profile=0))
