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
