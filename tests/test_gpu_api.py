"""C-ABI behaviour that needs live contexts (a GPU)."""
import pytest

import jp2hip

pytestmark = pytest.mark.gpu


def test_env_check_names_too_few_queues(monkeypatch):
    """jp2hip_env_check compares GPU_MAX_HW_QUEUES (read at the call) with the
    contexts alive in the process: three contexts on two queues are named,
    and the advice goes once the variable covers them."""
    encs = [jp2hip.Encoder(0) for _ in range(3)]
    try:
        monkeypatch.setenv("GPU_MAX_HW_QUEUES", "2")
        assert "GPU_MAX_HW_QUEUES=2" in jp2hip._lib.env_check()
        monkeypatch.setenv("GPU_MAX_HW_QUEUES", "32")
        assert jp2hip._lib.env_check() == ""
    finally:
        for e in encs:
            e.close()


def test_output_tail_reads_in_place():
    """Output.tail(k) (the bench's EOC check) equals the view's last bytes."""
    import imaging as im
    from devmem import DeviceBytes
    tif = im.tiff_bytes(im.synth_rgb8(200, 300, seed=4))
    lay, _ = jp2hip.tiff_layout(tif)
    d = DeviceBytes(tif)
    e = jp2hip.Encoder(0)
    try:
        out, _ = e.encode_device(d.ptr, d.nbytes, lay, jp2hip.LOSSY, jp2hip.recipe(jp2hip.LOSSY), copy=False)
        assert out.tail(2) == b"\xff\xd9"
        assert out.tail(10) == bytes(out.view()[-10:])
        out.close()
    finally:
        e.close()
        d.free()
