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


def golden_image(name, testjpx_pixels):
    """Source pixels of a tests/golden/golden.json "lossy" case, by name."""
    import imaging as im
    table = {
        "synth_rgb8_1024x1536": lambda: im.synth_rgb8(1024, 1536, seed=1234),
        "testjpx_rgb_crop_1024": lambda: testjpx_pixels[:1024, :1024, :3].copy(),
        "synth_gray16_1024": lambda: im.synth_u16(1024, 1024, comps=1, seed=5),
        "c2_synth_rgb8_6000x4000": lambda: im.synth_rgb8(4000, 6000, seed=1234),
        "c2_testjpx_tiled_6000x4000": lambda: im.testjpx_tiled(testjpx_pixels),
        "c5_gray16_4096x4096": lambda: im.synth_gray16_rows(0, 4096, 4096),
    }
    return table[name]()
