import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(ROOT, "tests", "golden")


# Run first: these put W rank processes on the box's one GPU, and while the
# test process holds no GPU context of its own yet they run faster (W + 1 > 8
# processes on one GPU: the W = 8 rehearsal at 8 x 100M took 31 s instead of
# 9 s, profiles/r06/rehearsal_context_probe.txt).  A speed-up only: the
# suite passes in any order (SFL_TEST_NO_REORDER=1 keeps pytest's own).
_FIRST = ("test_gpu_bench_rehearsal.py", "test_gpu_dist_pipeline.py", "test_gpu_rccl_multirank.py")


def pytest_collection_modifyitems(session, config, items):
    if os.environ.get("SFL_TEST_NO_REORDER") == "1":
        return
    first = [it for it in items if os.path.basename(str(it.fspath)) in _FIRST]
    if first:
        rest = [it for it in items if os.path.basename(str(it.fspath)) not in _FIRST]
        items[:] = first + rest
