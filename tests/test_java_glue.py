"""GpuConverter's native side without a JVM.

jp2-bucketeer_amd/java holds the Java converter, the reference-side patches
(ConverterFactory / ImageWorkerVerticle / MainVerticle / Config) and the JNI
natives, which are type conversions around jp2hip_glue.c.  No JDK exists in
this image, so what runs here is tests/host/glue_replay.c: the natives' exact
call sequence (probe -> ordinals -> create x N -> split_peers -> env_check ->
tiff_pixels -> encode_file -> last_error -> destroy, plus the failure paths)
on the same glue functions, built with AddressSanitizer (host code only)."""
import os
import re
import subprocess

import numpy as np
import pytest

import imaging as im

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JAVA = os.path.join(ROOT, "jp2-bucketeer_amd", "java")
REPLAY = os.path.join(JAVA, "build", "glue_replay_asan")
# the HIP runtime's own allocations are not ours to judge; the harness may
# preload a library ahead of the ASan runtime
SUPP = "leak:libamdhip64\nleak:libhsa-runtime64\nleak:libhsakmt\nleak:librocprofiler\nleak:libdrm\n"


def _replay_env(tmp_path):
    supp = tmp_path / "lsan.supp"
    supp.write_text(SUPP)
    env = dict(os.environ)
    env["ASAN_OPTIONS"] = "verify_asan_link_order=0:detect_leaks=1:abort_on_error=0"
    env["LSAN_OPTIONS"] = f"suppressions={supp}:print_suppressions=0"
    return env


def _build():
    subprocess.run(["make", "-s", "-C", JAVA, "replay"], check=True, capture_output=True, timeout=300)


def test_every_native_has_a_jni_function():
    java = open(os.path.join(JAVA, "src/main/java/edu/ucla/library/bucketeer/converters/GpuConverter.java")).read()
    jni = open(os.path.join(JAVA, "src/main/c/jp2hip_jni.c")).read()
    natives = re.findall(r"private static native \S+ (native\w+)\(", java)
    assert len(natives) >= 6
    for n in natives:
        assert f"Java_edu_ucla_library_bucketeer_converters_GpuConverter_{n}(" in jni, n
    # close() releases the contexts; a failed constructor leaves none (glue_open)
    assert "public void close()" in java and "nativeClose(myHandles)" in java


def test_patches_are_well_formed():
    """The reference-side patches are unified diffs of the four files a
    maintainer edits; each hunk's line counts match its body."""
    pdir = os.path.join(JAVA, "patches")
    names = sorted(os.listdir(pdir))
    assert names == ["Config.java.patch", "ConverterFactory.java.patch", "ImageWorkerVerticle.java.patch",
                     "MainVerticle.java.patch"]
    for n in names:
        lines = open(os.path.join(pdir, n)).read().splitlines()
        assert lines[0].startswith("--- a/src/main/java/") and lines[1].startswith("+++ b/src/main/java/")
        i = 2
        while i < len(lines):
            m = re.match(r"@@ -(\d+),(\d+) \+(\d+),(\d+) @@", lines[i])
            assert m, (n, lines[i])
            old, new = int(m.group(2)), int(m.group(4))
            i += 1
            while i < len(lines) and not lines[i].startswith("@@"):
                c = lines[i][:1]
                old -= c in (" ", "-")
                new -= c in (" ", "+")
                i += 1
            assert old == 0 and new == 0, n


@pytest.mark.skipif(not os.path.isdir("/root/reference/src"), reason="reference checkout not present")
def test_patches_apply_to_the_reference(tmp_path):
    import shutil
    for f in ("converters/ConverterFactory.java", "verticles/ImageWorkerVerticle.java",
              "verticles/MainVerticle.java", "Config.java"):
        src = os.path.join("/root/reference/src/main/java/edu/ucla/library/bucketeer", f)
        dst = tmp_path / "src/main/java/edu/ucla/library/bucketeer" / f
        dst.parent.mkdir(parents=True, exist_ok=True)
        shutil.copy(src, dst)
    for p in sorted(os.listdir(os.path.join(JAVA, "patches"))):
        r = subprocess.run(["patch", "-p1", "--dry-run", "-i", os.path.join(JAVA, "patches", p)], cwd=tmp_path,
                           capture_output=True, text=True)
        assert r.returncode == 0, r.stdout + r.stderr


def test_glue_replay_without_gpu_under_asan(tmp_path):
    """On a host without a gfx950 device: probe 0, the constructor fails
    cleanly (nothing allocated), create / encode report errors; ASan and
    LeakSanitizer find nothing in the host code."""
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a GPU is visible: the GPU test covers this host")
    except ImportError:
        pass
    _build()
    tif = tmp_path / "a.tif"
    tif.write_bytes(im.tiff_bytes(im.synth_rgb8(40, 50, seed=1)))
    p = subprocess.run([REPLAY, str(tmp_path), "1", "1", str(tif)], capture_output=True, text=True, timeout=120,
                       env=_replay_env(tmp_path))
    assert p.returncode == 0, p.stdout + p.stderr
    assert "probe 0" in p.stdout and f"tiff_pixels {tif} 2000" in p.stdout
    assert p.stdout.strip().endswith("REPLAY OK")
    assert "AddressSanitizer" not in p.stderr and "LeakSanitizer" not in p.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("conversion", [1, 0])
def test_glue_replay_on_gpu_under_asan(tmp_path, conversion):
    """The converter's whole native life on the GPU: pooled contexts, a split
    context (peer on the same device on a one-GPU box), 4 threads converting
    6 TIFFs (one of >= 3 MP through the split route), a constructor failing
    part-way and an out-of-range split ordinal (clean errors, no fault), a
    missing TIFF and an unwritable output (IOException text), close().  Every
    file equals the oracle's; the host code is clean under ASan."""
    import oracle_lib as ol
    _build()
    imgs, paths = [], []
    for i in range(6):
        img = im.synth_rgb8(300 + 41 * i, 280 + 29 * i, seed=60 + i) if i < 5 else im.synth_rgb8(1500, 2100, seed=66)
        p = tmp_path / f"in{i}_é.tif"  # a non-ASCII path (熵.tif in ImageUploadKakaduIT.java:69)
        p.write_bytes(im.tiff_bytes(img))
        imgs.append(img)
        paths.append(str(p))
    out = tmp_path / "out"
    out.mkdir()
    r = subprocess.run([REPLAY, str(out), str(conversion), "4"] + paths, capture_output=True, text=True,
                       timeout=300, env=_replay_env(tmp_path))
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert r.stdout.strip().endswith("REPLAY OK")
    assert "via split context: ok" in r.stdout and "via pooled context: ok" in r.stdout
    assert "create on ordinal 4096: rc -1" in r.stdout and "split_peers with ordinal 4096: rc -1" in r.stdout
    assert "contexts for memory 16" in r.stdout  # an idle MI355X: 288 GB x 0.75 / 8 GiB > 16
    assert "AddressSanitizer" not in r.stderr
    import jp2hip
    for i, img in enumerate(imgs):
        got = (out / f"out{i:03d}.jpx").read_bytes()
        assert got == ol.encode(img, ol.copy_recipe(jp2hip.recipe(conversion))), i
        if conversion == 1:
            assert np.array_equal(im.decode_pillow(got), img)
