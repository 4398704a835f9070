/* jp2hip_glue.c -- see jp2hip_glue.h.  Plain C99 over include/jp2hip.h. */
#include "jp2hip_glue.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "jp2hip.h"

static void set_err(char *err, size_t errlen, const char *prefix, const char *msg) {
    if (!err || !errlen) return;
    snprintf(err, errlen, "%s%s", prefix ? prefix : "", msg ? msg : "");
}

/* a Java byte[] path (UTF-8, no terminator) as a C string; NULL when out of memory */
static char *path_of(const char *p, size_t n) {
    char *s = (char *)malloc(n + 1);
    if (!s) return NULL;
    if (n) memcpy(s, p, n);
    s[n] = 0;
    return s;
}

int glue_probe(void) { return jp2hip_probe() ? 1 : 0; }

int glue_device_ordinals(int32_t *ordinals, int max) {
    int n = jp2hip_device_ordinals(ordinals, max);
    if (n < 0) n = 0;
    return n > max ? max : n;
}

const char *glue_env_check(void) {
    const char *s = jp2hip_env_check();
    return s ? s : "";
}

int glue_create(int device, int host_threads, int64_t *handle, char *err, size_t errlen) {
    jp2hip_config cfg;
    memset(&cfg, 0, sizeof cfg);
    cfg.device = device;
    cfg.host_threads = host_threads;
    jp2hip_ctx *ctx = NULL;
    *handle = 0;
    if (jp2hip_create(&ctx, &cfg) != 0) {
        char pre[64];
        snprintf(pre, sizeof pre, "GPU %d: ", device);
        set_err(err, errlen, pre, jp2hip_last_error());  /* thread-local: read on this thread */
        return -1;
    }
    *handle = (int64_t)(intptr_t)ctx;
    return 0;
}

int glue_split_peers(int64_t handle, const int32_t *ordinals, int n, int64_t min_pixels, char *err, size_t errlen) {
    if (jp2hip_split_peers((jp2hip_ctx *)(intptr_t)handle, ordinals, n, min_pixels) != 0) {
        set_err(err, errlen, "split context: ", jp2hip_last_error());
        return -1;
    }
    return 0;
}

int64_t glue_tiff_pixels(const char *path, size_t path_len) {
    char *p = path_of(path, path_len);
    if (!p) return -1;
    const int64_t n = jp2hip_tiff_pixels(p);
    free(p);
    return n < 0 ? -1 : n;
}

int glue_encode_file(int64_t handle, const char *tiff, size_t tiff_len, const char *out, size_t out_len,
                     int conversion, char *err, size_t errlen) {
    char *in_path = path_of(tiff, tiff_len), *out_path = path_of(out, out_len);
    int rc = -1;
    if (!in_path || !out_path) set_err(err, errlen, NULL, "out of memory");
    else if (jp2hip_encode_file((jp2hip_ctx *)(intptr_t)handle, in_path, out_path, conversion, NULL, NULL) == 0) rc = 0;
    else set_err(err, errlen, NULL, jp2hip_last_error());
    free(in_path);
    free(out_path);
    return rc;
}

void glue_destroy(int64_t handle) {
    if (handle) jp2hip_destroy((jp2hip_ctx *)(intptr_t)handle);
}

void glue_close(const int64_t *handles, int n, int64_t split) {
    for (int i = 0; i < n; i++) glue_destroy(handles[i]);
    glue_destroy(split);
}

int glue_contexts_for_memory(int device, int64_t budget, int cap) {
    int64_t fr = 0, tot = 0;
    if (budget <= 0) budget = GLUE_CONTEXT_BUDGET;
    if (jp2hip_device_memory(device, &fr, &tot) != 0) return 1;
    const int64_t k = (fr / 4 * 3) / budget;
    return k < 1 ? 1 : (k > cap ? cap : (int)k);
}

int glue_open(int per_gpu, int64_t split_min_pixels, int64_t *handles, int max_handles, int *n, int64_t *split,
              char *err, size_t errlen) {
    int32_t gpus[64];
    *n = 0;
    *split = 0;
    const int ng = glue_device_ordinals(gpus, 64);
    if (ng == 0) {
        set_err(err, errlen, NULL, "no gfx950 GPU visible");
        return -1;
    }
    if (per_gpu < 1) { /* from the devices' free memory: the smallest share of them */
        per_gpu = GLUE_MAX_CONTEXTS_PER_GPU;
        for (int g = 0; g < ng; g++) {
            const int k = glue_contexts_for_memory(gpus[g], 0, GLUE_MAX_CONTEXTS_PER_GPU);
            if (k < per_gpu) per_gpu = k;
        }
    }
    for (int slot = 0; slot < per_gpu; slot++)
        for (int g = 0; g < ng; g++) {
            if (*n >= max_handles) {
                set_err(err, errlen, NULL, "too many contexts for the handle table");
                goto fail;
            }
            if (glue_create(gpus[g], 0, &handles[*n], err, errlen) != 0) goto fail;
            (*n)++;
        }
    if (ng > 1) {
        if (glue_create(gpus[0], 0, split, err, errlen) != 0) goto fail;
        if (glue_split_peers(*split, gpus + 1, ng - 1, split_min_pixels, err, errlen) != 0) goto fail;
    }
    return 0;
fail:
    /* a constructor that fails releases what it made (GpuConverter.java) */
    glue_close(handles, *n, *split);
    *n = 0;
    *split = 0;
    return -1;
}
