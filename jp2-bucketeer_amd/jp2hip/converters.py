"""Host-side mirror of Bucketeer's converter plug-in API.

Reference (src/main/java/edu/ucla/library/bucketeer/converters/):
  Conversion.java:8-10        enum Conversion {LOSSY, LOSSLESS}
  Converter.java:10-24        File convert(String aID, File aTIFF, Conversion)
  KakaduConverter.java:26-128 kdu_compress wrapper (recipe :38-44, output name :57,
                              KAKADU_HOME :111-128)
  OpenJPEGConverter.java:9-27 stub, convert() returns null
  ConverterFactory.java:20-103 getConverter(), getConverter(Class), checkSystemKakadu()

``GpuConverter`` is the new plug-in: same contract as KakaduConverter.convert
(blocking, output ``<tmp>/<workdir>/<urlencoded id>.jpx`` owned by the caller,
every failure an ``IOError`` carrying the BUCKETEER-001 text), but the encode
runs in-process on MI355X through libjp2hip instead of a kdu_compress child.
"""
from __future__ import annotations

import enum
import logging
import os
import shutil
import subprocess
import tempfile
import threading
import urllib.parse
from pathlib import Path

from . import _lib

# bucketeer_messages.xml:12  BUCKETEER-001 "Failed to convert TIFF to JP2: {}"
BUCKETEER_001 = "Failed to convert TIFF to JP2: {}"
# BUCKETEER-002 (KakaduConverter.getPath, :97-103)
BUCKETEER_002 = "Output directory is not writable: {}"
# BUCKETEER-032 (ConverterFactory.getConverter(Class), :70)
BUCKETEER_032 = "No known converter"


class Conversion(enum.IntEnum):
    """Conversion.java:8-10 (ordinals kept: LOSSY=0, LOSSLESS=1)."""
    LOSSY = _lib.LOSSY
    LOSSLESS = _lib.LOSSLESS


class KakaduNotFoundError(RuntimeError):
    """KakaduNotFoundException (an unchecked I18nRuntimeException in the reference)."""


class Converter:
    """Converter.java:10-24."""

    def convert(self, image_id: str, tiff: os.PathLike | str, conversion: Conversion) -> Path:
        raise NotImplementedError


def _jpx_name(image_id: str) -> str:
    # URLEncoder.encode(aID, UTF-8) + ".jpx"   (KakaduConverter.java:57)
    return urllib.parse.quote_plus(image_id, safe="*-._") + ".jpx"


class KakaduConverter(Converter):
    """Mirror of KakaduConverter.java: shells out to kdu_compress with the recipe."""

    WORKING_DIR_NAME = "kakadu"
    KAKADU_HOME = "KAKADU_HOME"
    BASE_OPTIONS = ["Clevels=6", "Clayers=6", "Cprecincts={256,256},{256,256},{128,128}",
                    "Stiles={512,512}", "Corder=RPCL", "ORGgen_plt=yes", "ORGtparts=R",
                    "Cblk={64,64}", "Cuse_sop=yes", "Cuse_eph=yes", "-flush_period", "1024"]
    LOSSLESS_OPTIONS = ["Creversible=yes", "-rate", "-"]
    LOSSY_OPTION = ["-rate", "3"]

    def __init__(self):
        self.tmp_dir = Path(tempfile.gettempdir()) / self.WORKING_DIR_NAME
        self.tmp_dir.mkdir(parents=True, exist_ok=True)

    @classmethod
    def get_executable(cls) -> str:
        home = os.environ.get(cls.KAKADU_HOME)
        return str(Path(home) / "kdu_compress") if home else "kdu_compress"

    def convert(self, image_id, tiff, conversion):
        jpx = self.tmp_dir / _jpx_name(image_id)
        cmd = [self.get_executable(), "-i", str(Path(tiff).absolute()), "-o", str(jpx)]
        cmd += self.BASE_OPTIONS
        cmd += self.LOSSLESS_OPTIONS if conversion == Conversion.LOSSLESS else self.LOSSY_OPTION
        if not ConverterFactory.has_system_kakadu():
            raise KakaduNotFoundError("Kakadu not found")
        proc = subprocess.run(cmd, capture_output=True)
        if proc.returncode != 0:
            raise IOError(BUCKETEER_001.format(image_id))
        return jpx


class OpenJPEGConverter(Converter):
    """OpenJPEGConverter.java:9-27 -- the reference's stub; convert() returns None."""

    def convert(self, image_id, tiff, conversion):
        return None


class GpuConverter(Converter):
    """MI355X converter: libjp2hip in-process, a pool of contexts (images in
    flight) on every visible gfx950 device, plus one split context whose peers
    cover ``split_devices`` (default: every device, when there are several):
    an image of at least ``split_min_pixels`` (default 256 MP, or
    ``JP2HIP_SPLIT_MIN_PIXELS``) is tile-split across those GPUs inside
    jp2hip_encode_file (jp2hip_split_peers), a smaller one takes a pool
    context.

    Safe for concurrent callers (the reference runs one ImageWorkerVerticle
    thread, MainVerticle.java:229-231; raising that count gives each call its
    own GPU context from the pool; oversized images take turns on the split
    context).
    """

    WORKING_DIR_NAME = "jp2hip"
    SPLIT_MIN_PIXELS = 256_000_000

    def __init__(self, devices: list[int] | None = None, host_threads: int = 0, per_gpu: int | None = None,
                 split_devices: list[int] | None = None, split_min_pixels: int | None = None):
        self.tmp_dir = Path(tempfile.gettempdir()) / self.WORKING_DIR_NAME
        self._pool, self._free = [], []
        self._cv = threading.Condition()
        self._split, self._split_lock, self.split_world = None, threading.Lock(), 1
        self._closed = False
        self.unavailable = None  # reason every convert() fails with (GPU absent / init failed)
        try:
            self.tmp_dir.mkdir(parents=True, exist_ok=True)
        except OSError as e:  # KakaduConverter.java:48-52 throws BUCKETEER_163 here
            raise IOError(BUCKETEER_002.format(self.tmp_dir)) from e
        if devices is None:
            devices = _lib.device_ordinals()
        if split_devices is None:
            split_devices = list(devices) if len(devices) > 1 else []
        if split_min_pixels is None:
            split_min_pixels = int(os.environ.get("JP2HIP_SPLIT_MIN_PIXELS", self.SPLIT_MIN_PIXELS))
        self.split_min_pixels = split_min_pixels
        try:
            if per_gpu is None:  # as many as the devices' free memory holds (GpuConverter.java)
                per_gpu = min(_lib.contexts_for_memory(_lib.device_memory(d)[0]) for d in devices) if devices else 1
            self.per_gpu = per_gpu
            self._pool = [_lib.Encoder(d, host_threads) for _ in range(max(1, per_gpu)) for d in devices]
            if len(split_devices) > 1:
                self._split = _lib.Encoder(split_devices[0], host_threads)
                self._split.split_peers(list(split_devices[1:]), split_min_pixels)
                self.split_world = len(split_devices)
        except _lib.Jp2hipError as e:
            self.close()
            self._pool = []
            raise IOError(BUCKETEER_001.format(f"(GPU converter init: {e})")) from e
        if not self._pool:
            raise IOError(BUCKETEER_001.format("(no gfx950 device)"))
        self._free = list(self._pool)
        # the slow configurations the library can see (queues, SDMA): logged once
        self.env_advice = _lib.env_check()
        if self.env_advice:
            logging.getLogger(__name__).warning("libjp2hip: %s", self.env_advice)

    @classmethod
    def unavailable_converter(cls, reason: str) -> "GpuConverter":
        """A GpuConverter whose convert() raises IOError(BUCKETEER_001 ...):
        what ConverterFactory hands out when the GPU cannot be used and Kakadu
        is absent, so ImageWorkerVerticle's IOException handler (:106) answers
        the event-bus message instead of an unchecked exception escaping it."""
        c = cls.__new__(cls)
        c.tmp_dir = Path(tempfile.gettempdir()) / cls.WORKING_DIR_NAME
        c._pool, c._free, c._cv = [], [], threading.Condition()
        c._split, c._split_lock, c.split_world = None, threading.Lock(), 1
        c._closed = False
        c.unavailable = reason
        return c

    def _acquire(self, image_id):
        # waiters see close() at once (a borrower must get the
        # IOError, not block on a pool that close() is draining)
        with self._cv:
            while not self._free and not self._closed:
                self._cv.wait()
            if self._closed:
                raise IOError(BUCKETEER_001.format(image_id) + ": converter closed")
            return self._free.pop()

    def _release(self, enc):
        with self._cv:
            self._free.append(enc)
            self._cv.notify_all()

    def convert(self, image_id, tiff, conversion):
        if self.unavailable is not None:
            raise IOError(BUCKETEER_001.format(image_id) + f": {self.unavailable}")
        tiff = Path(tiff)
        jpx = self.tmp_dir / _jpx_name(image_id)
        if not os.access(jpx.parent, os.W_OK):
            raise IOError(BUCKETEER_002.format(jpx))
        if self._closed:
            raise IOError(BUCKETEER_001.format(image_id) + ": converter closed")
        try:
            big = self._split is not None and _lib.tiff_pixels(str(tiff.absolute())) >= self.split_min_pixels
            if big:
                # split encodes take turns with each other only: the pool's
                # condition (_cv) is never held across an encode, so pooled
                # conversions go on while an oversized image holds every GPU
                with self._split_lock:
                    if self._closed or self._split is None:
                        raise IOError(BUCKETEER_001.format(image_id) + ": converter closed")
                    self._split.encode_file(str(tiff.absolute()), str(jpx), int(Conversion(conversion)))
                return jpx
            enc = self._acquire(image_id)
            try:
                enc.encode_file(str(tiff.absolute()), str(jpx), int(Conversion(conversion)))
            finally:
                self._release(enc)
        except (_lib.Jp2hipError, ValueError) as e:
            raise IOError(BUCKETEER_001.format(image_id) + f": {e}") from e
        return jpx

    def close(self):
        """Later conversions (and borrowers still waiting) fail with IOError;
        conversions in progress finish first, then every context is released
        (GpuConverter.java close())."""
        with self._cv:
            self._closed = True
            self._cv.notify_all()
            while len(self._free) < len(self._pool):
                self._cv.wait()
            pool, self._pool, self._free = self._pool, [], []
        for e in pool:
            e.close()
        with self._split_lock:
            if self._split is not None:
                self._split.close()
                self._split = None


class ConverterFactory:
    """ConverterFactory.java:20-103, plus the GPU branch."""

    _converter: Converter | None = None
    _has_kakadu = False
    _lock = threading.Lock()
    _closing: list[threading.Thread] = []

    @classmethod
    def get_converter(cls, klass: type | None = None) -> Converter:
        with cls._lock:
            if klass is None:
                # exactly the reference's rule (ConverterFactory.java:37-47):
                # Kakadu if present, else OpenJPEG. The GPU is chosen only by
                # name (get_converter(GpuConverter), the bucketeer.converter
                # key), so KakaduConverterTest.java:99's cast still holds on a
                # host with Kakadu and a gfx950 device.
                if cls._converter is None:
                    if cls.check_system_kakadu():
                        cls._converter = KakaduConverter()
                    else:
                        cls._converter = OpenJPEGConverter()
                return cls._converter
            if klass is KakaduConverter:
                if not cls.check_system_kakadu():
                    raise KakaduNotFoundError("Kakadu not found")
                cls._replace(KakaduConverter())
            elif klass is OpenJPEGConverter:
                cls._replace(OpenJPEGConverter())
            elif klass is GpuConverter:
                # never raises: GPU if usable, else Kakadu if present, else a
                # converter whose convert() raises IOError (the caller's
                # handler, ImageWorkerVerticle.java:106, catches only that)
                if not (isinstance(cls._converter, GpuConverter) and cls._converter.unavailable is None):
                    reason = "no gfx950 device"
                    conv = None
                    if cls.check_system_gpu():
                        try:
                            conv = GpuConverter()
                        except IOError as e:
                            reason = str(e)
                    if conv is None:
                        conv = KakaduConverter() if cls.check_system_kakadu() else \
                            GpuConverter.unavailable_converter(reason)
                    cls._replace(conv)
            else:
                raise ValueError(BUCKETEER_032)
            return cls._converter

    @classmethod
    def _replace(cls, conv: Converter):
        """Install ``conv`` as the singleton; a GpuConverter it displaces is
        closed on a thread of its own (close() waits for the conversions in
        progress, which must not hold the factory lock), so its contexts are
        released instead of leaked."""
        old, cls._converter = cls._converter, conv
        if isinstance(old, GpuConverter) and old is not conv:
            t = threading.Thread(target=old.close, name="GpuConverter-close", daemon=True)
            t.start()
            cls._closing.append(t)

    @classmethod
    def has_system_kakadu(cls) -> bool:
        return cls._has_kakadu

    @classmethod
    def check_system_kakadu(cls) -> bool:
        """`kdu_compress -v` exit status (ConverterFactory.java:86-103)."""
        exe = KakaduConverter.get_executable()
        ok = False
        if shutil.which(exe) or os.path.exists(exe):
            try:
                ok = subprocess.run([exe, "-v"], capture_output=True).returncode == 0
            except OSError:
                ok = False
        cls._has_kakadu = ok
        return ok

    @classmethod
    def check_system_gpu(cls) -> bool:
        try:
            return _lib.probe()
        except _lib.Jp2hipError:
            return False

    @classmethod
    def reset(cls):
        with cls._lock:
            if isinstance(cls._converter, GpuConverter):
                cls._converter.close()
            cls._converter = None
            closing, cls._closing = cls._closing, []
        for t in closing:
            t.join()
