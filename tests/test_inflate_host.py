"""k_inflate (kernels.hip) compiled for the host -- a one-lane wave -- and run under AddressSanitizer:
zlib streams of every level at every byte alignment decode exactly, and
truncated or reserved-block streams report a corrupt strip.  The GPU tests
(test_gpu_parity.py) run the same kernel on the device; this one runs on CPU."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(__file__)
SRC = os.path.join(HERE, "..", "jp2-bucketeer_amd", "csrc", "kernels.hip")
HDR = os.path.join(HERE, "..", "jp2-bucketeer_amd", "csrc", "gpu_encoder.h")
CLANG = "/opt/rocm/llvm/bin/clang++"


def _kernel_text():
    h = open(HDR).read()
    ua = h[h.index("struct UnpackArgs {"):h.index("// LZW strips, segment-parallel")]
    s = open(SRC).read()
    inf = s[s.index("#ifndef JP2HIP_INF_LANES"):s.index("// Predictor 2: each sample adds")]
    return "namespace jp2hip {\n" + ua + inf + "}\n"


@pytest.mark.skipif(not os.path.exists(CLANG) or not os.path.exists("/usr/include/zlib.h"),
                    reason="needs ROCm clang++ and zlib headers")
def test_inflate_host_build(tmp_path):
    main = open(os.path.join(HERE, "host", "inflate_main.cpp")).read()
    shims, rest = main.split("// [[MAIN]]")
    src = tmp_path / "inflate_host.cpp"
    src.write_text(shims + _kernel_text() + rest)
    exe = tmp_path / "inflate_host"
    subprocess.run([CLANG, "-O1", "-g", "-std=c++17", "-fsanitize=address", str(src), "-o", str(exe), "-lz"],
                   check=True, capture_output=True, timeout=240)
    p = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    assert p.stdout.strip().endswith("OK")
