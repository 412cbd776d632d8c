import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: longer-running CPU test")


@pytest.fixture(scope="session")
def native():
    import distributed_cuda_bfs_amd as dbfs
    return dbfs.native


@pytest.fixture(scope="session")
def data_dir():
    return os.path.join(REPO, "tests", "data")


@pytest.fixture(scope="session")
def gpu_runtime():
    """Single-rank HIP runtime (fails loudly when no GPU is visible)."""
    import distributed_cuda_bfs_amd as dbfs
    from distributed_cuda_bfs_amd.parallel.runtime import init_runtime
    if dbfs.native.hip_device_count() < 1:
        pytest.fail("gpu test selected but no HIP device is visible")
    return init_runtime("hip")
