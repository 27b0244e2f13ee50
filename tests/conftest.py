import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")
    config.addinivalue_line("markers", "slow: long-running end-to-end test")
    # Build the native core once per session (no-op when up to date).
    from p2p_llm_tunnel_amd.utils.build import ensure_native
    ensure_native()


@pytest.fixture(scope="session")
def native():
    from p2p_llm_tunnel_amd import native as _n
    return _n()


@pytest.fixture
def mock_upstream():
    from p2p_llm_tunnel_amd.utils import mock_llm
    srv, port = mock_llm.start_in_thread(threaded=True)
    yield f"http://127.0.0.1:{port}"
    srv.shutdown()
    srv.server_close()
