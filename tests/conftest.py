import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "jp2-bucketeer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def testjpx_bytes():
    with open(os.path.join(GOLDEN, "test.jpx"), "rb") as f:
        return f.read()


@pytest.fixture(scope="session")
def testjpx_pixels(testjpx_bytes):
    """Decoded pixels of the reference's only image fixture (the C1 source proxy)."""
    import imaging
    return imaging.decode_pillow(testjpx_bytes)


@pytest.fixture(scope="session")
def encoder():
    import jp2hip
    enc = jp2hip.Encoder(0)
    yield enc
    enc.close()
