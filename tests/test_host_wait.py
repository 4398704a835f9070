"""The bounded host wait of the code-stream copy (csrc/host_wait.h, used by
t2_device.hip dma_to_host): compiled with g++ and run on the CPU, under
AddressSanitizer/UBSan."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_wait_bounded_on_cpu(tmp_path):
    exe = tmp_path / "test_host_wait"
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-Wall", "-Wextra", "-Werror",
                    "-I", os.path.join(ROOT, "jp2-bucketeer_amd", "csrc"),
                    os.path.join(ROOT, "tests", "host", "test_host_wait.cpp"), "-o", str(exe)],
                   check=True, capture_output=True, timeout=300)
    env = dict(os.environ, ASAN_OPTIONS="verify_asan_link_order=0:detect_leaks=0")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().endswith("HOST WAIT OK")


def test_dma_to_host_has_no_unbounded_wait():
    src = open(os.path.join(ROOT, "jp2-bucketeer_amd", "csrc", "t2_device.hip")).read()
    assert "UINT64_MAX" not in src
    assert src.count("jp2hip::wait_bounded(") >= 2  # the code-stream copy and the engine probe


def test_memory_policy_on_cpu(tmp_path):
    """The release-after-encode rule (csrc/mem_policy.h, used by api.cpp's
    EncodeEnd): keep a steady large footprint, release after an outsized
    image, an explicit soft limit wins."""
    exe = tmp_path / "test_mem_policy"
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-Wall", "-Wextra", "-Werror",
                    "-I", os.path.join(ROOT, "jp2-bucketeer_amd", "csrc"),
                    os.path.join(ROOT, "tests", "host", "test_mem_policy.cpp"), "-o", str(exe)],
                   check=True, capture_output=True, timeout=300)
    env = dict(os.environ, ASAN_OPTIONS="verify_asan_link_order=0:detect_leaks=0")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().endswith("MEM POLICY OK")
