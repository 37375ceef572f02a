import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: larger CPU cases")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Compile the engine (hipcc cross-compiles without a GPU) and the oracle once."""
    from oversim_amd import build
    if os.environ.get("OVS_SKIP_BUILD") != "1":
        build.build_engine()
        build.build_oracle()
    yield


@pytest.fixture()
def engine():
    from oversim_amd import KbrEngine   # kbr.lib() imports torch first: one HIP runtime
    eng = KbrEngine(0)
    yield eng
    eng.close()
