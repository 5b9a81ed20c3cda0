import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "fs-dkr_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)
# the collect() pipeline runs up to eleven concurrent streams (see bench.py)
os.environ["GPU_MAX_HW_QUEUES"] = str(max(12, int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run via gpurun)")
    config.addinivalue_line("markers", "slow: long CPU test")


@pytest.fixture(scope="session")
def gpu_ctx():
    from fsdkr import Context
    ctx = Context(timing=True)
    yield ctx
    ctx.close()


@pytest.fixture(autouse=True)
def _whole_chip(request):
    """Each test starts on the whole chip: a shard test's GA CU split
    (shard.verify_slice -> fsdkr_ctx_set_cu_split) stays on the shared context,
    and tests that drive prestart / prepare directly (not refresh.collect, which
    resets it) would otherwise inherit it."""
    if "gpu_ctx" in request.fixturenames:
        request.getfixturevalue("gpu_ctx").set_cu_split(0)
    yield
