"""pytest configuration: `gpu` marker, import paths, shared fixtures.

CPU tests (-m "not gpu") cover the oracle against the golden vectors, the host build of the product's
device headers, the C-ABI surface of libat2v.so and the multi-rank (gloo) verdict plumbing.
GPU tests (-m gpu) are the parity tests proper: they call libat2v.so through its C ABI on a gfx950.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# The library reads its test / A-B environment hooks (AT2V_TEST_DEVICE_ALIAS, AT2V_TEST_FAIL_LAUNCH, ...) only in a
# process that sets this gate (csrc/at2v_env.h); the suite is such a process, a production node is not.
os.environ["AT2V_TEST_HOOKS"] = "1"
for p in (ROOT, os.path.join(ROOT, "at2-node_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (parity tests through the C ABI)")
    config.addinivalue_line("markers", "clean_gpu: multi-process latency test (no ordering: since round 5 a latency-mode "
                            "queue maps two hardware queues, and its p99 holds with other GPU processes around)")


@pytest.fixture(scope="session")
def oracle():
    import oracle_py
    return oracle_py.Oracle()


@pytest.fixture(scope="session")
def golden():
    import golden_io
    return golden_io.load_all()
