import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT / "reductionist-rs_amd", ROOT, ROOT / "tests"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device; run on the GPU box")


@pytest.fixture(scope="session")
def engine():
    """The product engine.  No CPU fallback: constructing it without a device raises."""
    from reductionist_amd import Engine
    return Engine()


@pytest.fixture(scope="session")
def workspace(engine):
    """A device-resident-path workspace (rdx_workspace) of the session engine."""
    ws = engine.workspace(0)
    yield ws
    ws.close()
