import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O

    O.build()  # incremental (make): picks up edits to oracle/*.c
    return O


@pytest.fixture(scope="session")
def native():
    from addapt_amd import native as N

    N.lib()  # fails loudly if the engine was not built
    return N
