import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle.oracle import OracleLib

    return OracleLib()


@pytest.fixture(scope="session")
def ref_golden():
    import numpy as np

    return np.load(ROOT / "tests" / "golden" / "reference_golden.npz")


@pytest.fixture(scope="session")
def ref_meta():
    import json

    return json.loads((ROOT / "tests" / "golden" / "reference_golden.json").read_text())


@pytest.fixture(scope="session")
def scipy_golden():
    import numpy as np

    return np.load(ROOT / "tests" / "golden" / "scipy_golden.npz")
