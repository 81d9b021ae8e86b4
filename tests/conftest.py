import sys
from pathlib import Path

import pytest

# torch (used by a few GPU tests for device buffers) ships its own HIP runtime; loading it before
# libmpcq.so makes both share one runtime (the dynamic linker reuses the loaded libamdhip64 SONAME).
import torch  # noqa: F401,E402

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device; run with -m gpu")


@pytest.fixture(scope="session")
def plant():
    from solvempc_amd import workload

    return workload.reference_plant()


@pytest.fixture(scope="session")
def golden_dir():
    return ROOT / "tests" / "golden"
