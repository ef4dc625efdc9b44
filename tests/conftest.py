import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT / "reductionist-rs_amd", ROOT, ROOT / "tests"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device; run on the GPU box")


def pytest_collection_modifyitems(session, config, items):
    """The BASELINE.json configs (C1-C5, `test_c<N>_*`) run first, so an `-x` stop in any other test
    cannot hide them; everything else keeps its collection order."""
    def key(item):
        name = item.name
        return (0, name) if len(name) > 6 and name.startswith("test_c") and name[6].isdigit() else (1, "")
    items.sort(key=key)   # stable: the second group keeps its order


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
