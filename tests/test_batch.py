"""Batch path: CSV -> per-GPU native queue
-> JPX + upload stand-in.

CPU tests cover the CSV mirror (JobFactory.java header rules), the sharding
and the output naming; GPU tests run the native queue (csrc/batch.cpp) and
compare every JPX byte for byte with the oracle, check the upload hook and
delete-after-upload (S3BucketVerticle.java:286-303), and that one bad row
fails alone (ImageWorkerVerticle.java:104-107 replies failure, the batch goes
on).
"""
import os

import numpy as np
import pytest

import imaging as im
import jp2hip
from jp2hip import batch as jb


def _write_csv(path, rows, header=("Item ARK", "Title", "File Name")):
    import csv
    with open(path, "w", newline="", encoding="utf-8") as f:
        w = csv.writer(f)
        w.writerow(header)
        w.writerows(rows)


def test_read_batch_csv_columns_and_empty_rows(tmp_path):
    p = tmp_path / "job.csv"
    _write_csv(p, [("ark:/21198/a1", "one", "a.tif"), ("ark:/21198/a2", "two", ""),
                   ("ark:/21198/熵", "three", "sub/b.tif")])
    items = jb.read_batch_csv(p, path_prefix="/data")
    assert [(i.job, i.image_id, i.tiff) for i in items] == [
        (0, "ark:/21198/a1", "/data/a.tif"), (2, "ark:/21198/熵", "/data/sub/b.tif")]


@pytest.mark.parametrize("header", [("Item ARK", "File Name", "File Name"), ("Title", "File Name"),
                                    ("Item ARK", "Item ARK", "File Name")])
def test_read_batch_csv_rejects_bad_headers(tmp_path, header):
    p = tmp_path / "bad.csv"
    _write_csv(p, [tuple("x" for _ in header)], header=header)
    with pytest.raises(jb.CsvError):
        jb.read_batch_csv(p)


def test_shard_is_a_partition():
    items = list(range(103))
    parts = [jb.shard(items, r, 8) for r in range(8)]
    assert sorted(x for p in parts for x in p) == items
    assert max(map(len, parts)) - min(map(len, parts)) <= 1


def test_jpx_name_matches_kakadu_converter():
    # KakaduConverter.java:57 URLEncoder.encode(id, UTF-8) + ".jpx"
    assert jb.jpx_name("ark:/21198/zz0001") == "ark%3A%2F21198%2Fzz0001.jpx"


def test_batch_structs_match_header():
    import ctypes
    txt = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include",
                            "jp2hip.h")).read()
    assert "jp2hip_batch_result" in txt
    assert ctypes.sizeof(jb.BatchConfig) == 8 * 4
    assert ctypes.sizeof(jb.BatchResult) == 8 + 4 + 4 + 3 * 8 + 3 * 8 + 240
    for sym in jb.BATCH_EXPORTS:
        assert hasattr(jp2hip._lib.lib(), sym)


@pytest.mark.gpu
def test_batch_queue_converts_uploads_and_deletes(tmp_path):
    import oracle_lib as ol
    src = tmp_path / "src"
    src.mkdir()
    imgs = {}
    rows = []
    for i in range(7):
        img = im.synth_rgb8(300 + 37 * i, 420 - 23 * i, seed=100 + i)
        name = f"img{i}.tif"
        (src / name).write_bytes(im.tiff_bytes(img, rows_per_strip=16 + i))
        imgs[f"ark:/21198/t{i}"] = img
        rows.append((f"ark:/21198/t{i}", f"t{i}", name))
    rows.append(("ark:/21198/missing", "gone", "nope.tif"))
    _write_csv(tmp_path / "job.csv", rows)
    items = jb.read_batch_csv(tmp_path / "job.csv", path_prefix=str(src))
    uploaded = {}

    def upload(image_id, path):  # S3 stand-in: keep the bytes, succeed
        with open(path, "rb") as f:
            uploaded[image_id] = f.read()
        return True

    res = jb.run_batch(items, tmp_path / "out", contexts=3, reader_threads=2, uploader_threads=2,
                       upload=upload)
    assert len(res) == len(items)
    by_job = {r["job"]: r for r in res}
    for it in items:
        r = by_job[it.job]
        if it.image_id.endswith("missing"):
            assert r["status"] == jb.CONVERT_FAILED and "cannot read TIFF" in r["message"]
            continue
        assert r["status"] == jb.OK, r["message"]
        got = uploaded[it.image_id]
        img = imgs[it.image_id]
        assert r["pixels"] == img.shape[0] * img.shape[1] and r["out_bytes"] == len(got)
        assert got == ol.encode(img, ol.recipe(True))
        # derivative image: deleted after the upload
        assert not (tmp_path / "out" / jb.jpx_name(it.image_id)).exists()


@pytest.mark.gpu
def test_batch_upload_failure_is_reported_and_file_kept(tmp_path):
    img = im.synth_rgb8(128, 160, seed=9)
    p = tmp_path / "a.tif"
    p.write_bytes(im.tiff_bytes(img))
    with jb.BatchQueue(contexts=1, upload=lambda iid, path: False) as q:
        q.submit(5, "ark:/x/fail", p, tmp_path / "a.jpx")
        res = q.drain()
    assert res[0]["job"] == 5 and res[0]["status"] == jb.UPLOAD_FAILED
    assert (tmp_path / "a.jpx").exists()  # S3BucketVerticle only deletes after success


@pytest.mark.gpu
def test_batch_compressed_tiff_with_many_strips(tmp_path):
    """An LZW TIFF with 600 one-row strips needs 1200 offset slots (offsets +
    byte counts); the reader sizes its retry from the strip count."""
    import oracle_lib as ol
    img = im.synth_rgb8(600, 96, seed=21)
    p = tmp_path / "many.tif"
    p.write_bytes(im.tiff_bytes_compressed(img, "tiff_lzw", rows_per_strip=1))
    with jb.BatchQueue(contexts=1) as q:
        q.submit(1, "ark:/x/many", p, tmp_path / "many.jpx")
        res = q.drain()
    assert res[0]["status"] == jb.OK, res[0]["message"]
    assert res[0]["pixels"] == 600 * 96


@pytest.mark.gpu
def test_batch_c4_full_size_image_identical_to_oracle(tmp_path, golden):
    """C4 at its configured size: one 5000x7000 RGB8 TIFF through the native
    batch queue (read, lossless encode, JPX write, stub upload) -- the file
    is the oracle's, byte for byte (golden SHA-256 from make_golden.py)."""
    import hashlib
    g = golden["lossless"][0]
    img = im.synth_rgb8(7000, 5000, seed=0)
    p = tmp_path / "c4.tif"
    p.write_bytes(im.tiff_bytes(img, rows_per_strip=64))
    got = {}

    def upload(image_id, path):
        with open(path, "rb") as f:
            got[image_id] = f.read()
        return True

    with jb.BatchQueue(contexts=2, upload=upload) as q:
        q.submit(1, "ark:/99999/synth00000", p, tmp_path / "c4.jpx")
        res = q.drain()
    assert res[0]["status"] == jb.OK, res[0]["message"]
    data = got["ark:/99999/synth00000"]
    assert len(data) == g["oracle_bytes"]
    assert hashlib.sha256(data).hexdigest() == g["oracle_sha256"]
    assert not (tmp_path / "c4.jpx").exists()


@pytest.mark.gpu
def test_batch_work_stealing_two_queues_on_the_gpu(tmp_path):
    """run_batch_dynamic over two native queues (one process, the pull model
    an N-GPU host uses; here both on device 0): mixed sizes, every row
    converted once, every file the oracle's, both queues used."""
    import oracle_lib as ol
    src = tmp_path / "src"
    src.mkdir()
    imgs, rows = {}, []
    for i in range(10):
        big = i % 4 == 0
        img = im.synth_rgb8(1100 if big else 200 + 13 * i, 900 if big else 260 - 7 * i, seed=300 + i)
        (src / f"m{i}.tif").write_bytes(im.tiff_bytes(img))
        imgs[f"ark:/21198/m{i}"] = img
        rows.append((f"ark:/21198/m{i}", f"m{i}", f"m{i}.tif"))
    _write_csv(tmp_path / "job.csv", rows)
    items = jb.read_batch_csv(tmp_path / "job.csv", path_prefix=str(src))
    uploaded, mu = {}, __import__("threading").Lock()

    def upload(image_id, path):
        with open(path, "rb") as f, mu:
            uploaded[image_id] = f.read()
        return True

    trace = []
    with jb.BatchQueue(contexts=2, reader_threads=1, uploader_threads=1, upload=upload) as q0, \
            jb.BatchQueue(contexts=2, reader_threads=1, uploader_threads=1, upload=upload) as q1:
        res = jb.run_batch_dynamic(items, tmp_path / "out", [q0, q1], depth=2, trace=trace)
    assert sorted(r["job"] for r in res) == [it.job for it in items]
    assert all(r["status"] == jb.OK for r in res), [r["message"] for r in res]
    assert {q for _, q, ev, _ in trace if ev == "submit"} == {0, 1}
    for iid, img in imgs.items():
        assert uploaded[iid] == ol.encode(img, ol.recipe(True)), iid
