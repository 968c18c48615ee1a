import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (gfx950) device and libpcabi.so')


@pytest.fixture(scope='session')
def oracle():
    """The CPU oracle (oracle/liboracle.so), built on demand. Test infrastructure only."""
    from tests import oracle_lib
    return oracle_lib.load()


@pytest.fixture(scope='session')
def gpu_lib():
    import torch  # noqa: F401  (one HIP runtime per process, see custom_porechop_abi_amd/_lib.py)
    from custom_porechop_abi_amd import _lib
    L = _lib.lib()
    if L.pcabi_device_count() < 1:
        pytest.fail('no HIP device visible but test is marked gpu')
    return L


@pytest.fixture(scope='session', autouse=True)
def _built_library():
    """libpcabi.so is a build artefact (git-ignored): build it once if this tree lacks it."""
    so = os.path.join(ROOT, 'custom_porechop_abi_amd', 'libpcabi.so')
    if not os.path.isfile(so):
        import __graft_entry__
        __graft_entry__.build_lib()
    yield
