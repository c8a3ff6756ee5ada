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


# Run first: these put W rank processes on the box's one GPU, so the test
# process must not hold a GPU context of its own yet (W + 1 processes at
# W = 8 is the suspected cause of rehearsals running ~10x slower, DESIGN.md
# §5); these modules never initialise HIP in the test process themselves.
_FIRST = ("test_gpu_bench_rehearsal.py", "test_gpu_dist_pipeline.py", "test_gpu_rccl_multirank.py")


def pytest_collection_modifyitems(session, config, items):
    first = [it for it in items if os.path.basename(str(it.fspath)) in _FIRST]
    if first:
        rest = [it for it in items if os.path.basename(str(it.fspath)) not in _FIRST]
        items[:] = first + rest
