/*
 * jp2hip_glue.h -- the native half of Bucketeer's GpuConverter, in plain C.
 *
 * GpuConverter.java's native methods (jp2hip_jni.c) are one-line JNI
 * wrappers over these functions: the JNI file only converts Java types
 * (byte[] paths, int[] ordinals, long handles, IOException).  Everything
 * else -- UTF-8 path handling, reading jp2hip_last_error() on the calling
 * thread, releasing what a failed constructor already created -- lives here,
 * so the exact call sequence the converter makes can be replayed without a
 * JVM (tests/host/glue_replay.c, run by tests/test_java_glue.py).
 *
 * Reference interfaces (src/main/java/edu/ucla/library/bucketeer/):
 *   converters/ConverterFactory.java:86-103  checkSystemKakadu()  -> glue_probe
 *   converters/KakaduConverter.java:48-52    new KakaduConverter() -> glue_open
 *   converters/Converter.java:22             convert()             -> glue_encode_file
 *   converters/AbstractConverter.java:33-35  stderr on failure     -> glue_encode_file's message
 */
#ifndef JP2HIP_GLUE_H
#define JP2HIP_GLUE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GLUE_ERR_LEN 512

/* ConverterFactory.checkSystemKakadu() analogue: 1 if a gfx950 device is usable. */
int glue_probe(void);

/* The gfx950 HIP ordinals (at most max), count returned (0: none). */
int glue_device_ordinals(int32_t *ordinals, int max);

/* "" or the environment advice (GPU_MAX_HW_QUEUES); never NULL. */
const char *glue_env_check(void);

/* One context on `device`; 0 and *handle set, or -1 with `err` filled. */
int glue_create(int device, int host_threads, int64_t *handle, char *err, size_t errlen);

/* Peers for the split context; 0 or -1 with `err`. */
int glue_split_peers(int64_t handle, const int32_t *ordinals, int n, int64_t min_pixels, char *err, size_t errlen);

/* Width x height of a TIFF (path as UTF-8 bytes, not NUL-terminated), or -1. */
int64_t glue_tiff_pixels(const char *path, size_t path_len);

/* Converter.convert(): 0, or -1 with jp2hip_last_error() of this thread in
 * `err` (paths as UTF-8 bytes of the given lengths: a Java byte[]). */
int glue_encode_file(int64_t handle, const char *tiff, size_t tiff_len, const char *out, size_t out_len,
                     int conversion, char *err, size_t errlen);

/* Releases a context (0 is ignored). */
void glue_destroy(int64_t handle);

/* What one pooled context is budgeted to hold (a C4-class 5000 x 7000 RGB8
 * lossless image; DESIGN.md 3 "Footprint"), and the pool's ceiling. */
#define GLUE_CONTEXT_BUDGET ((int64_t)8 << 30)
#define GLUE_MAX_CONTEXTS_PER_GPU 16

/* Contexts per GPU that fit 75 % of `device`'s free memory at `budget`
 * bytes each (<= 0: GLUE_CONTEXT_BUDGET), between 1 and `cap`. */
int glue_contexts_for_memory(int device, int64_t budget, int cap);

/* The whole GpuConverter constructor (GpuConverter.java): `per_gpu`
 * (<= 0: glue_contexts_for_memory of the device with the least free memory)
 * contexts on every gfx950 device (slot-major, as the Java pool fills), and
 * on a multi-GPU host one more context on the first device whose peers are
 * the others (the tile-split of oversized images).  On failure everything
 * created so far is destroyed and -1 returned with `err`; on success
 * handles[0 .. *n) are the pooled contexts and *split the split context (0 on
 * one GPU).  `handles` has room for max_handles. */
int glue_open(int per_gpu, int64_t split_min_pixels, int64_t *handles, int max_handles, int *n, int64_t *split,
              char *err, size_t errlen);

/* GpuConverter.close(): destroys the pooled and split contexts. */
void glue_close(const int64_t *handles, int n, int64_t split);

#ifdef __cplusplus
}
#endif
#endif
