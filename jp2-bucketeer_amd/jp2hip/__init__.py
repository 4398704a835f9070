"""jp2hip -- MI355X JPEG 2000 encoder behind Bucketeer's converter API.

``jp2hip.converters`` mirrors src/main/java/edu/ucla/library/bucketeer/converters;
``jp2hip._lib`` binds the C ABI of libjp2hip (include/jp2hip.h).
"""
from ._lib import (FORMAT_J2K, FORMAT_JP2, FORMAT_JPX, LOSSLESS, LOSSY, Encoder, Jp2hipError, Output,
                   device_count, device_ordinals, probe, recipe, tiff_layout, version)
from .converters import (Conversion, Converter, ConverterFactory, GpuConverter,
                         KakaduConverter, KakaduNotFoundError, OpenJPEGConverter)

__all__ = ["Conversion", "Converter", "ConverterFactory", "GpuConverter", "KakaduConverter",
           "KakaduNotFoundError", "OpenJPEGConverter", "Encoder", "Jp2hipError", "LOSSY",
           "LOSSLESS", "FORMAT_J2K", "FORMAT_JP2", "FORMAT_JPX", "Output", "device_count", "device_ordinals",
           "probe", "recipe", "tiff_layout", "version"]
