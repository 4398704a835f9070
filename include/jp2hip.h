/*
 * jp2hip.h -- C ABI of libjp2hip, the MI355X (gfx950) JPEG 2000 encoder that
 * replaces `kdu_compress` behind Bucketeer's converter plug-in API.
 *
 * Reference interfaces this ABI stands in for (paths relative to
 * src/main/java/edu/ucla/library/bucketeer/ in UCLALibrary/jp2-bucketeer):
 *
 *   converters/Converter.java:22
 *       File convert(String aID, File aTIFF, Conversion aConversion)
 *           -> jp2hip_encode_file(): TIFF path in, JPX path out, blocking,
 *              every failure reported as rc < 0 + jp2hip_last_error()
 *              (the Java side turns that into IOException, like
 *              AbstractConverter.java:33-35 does for a non-zero exit).
 *   converters/Conversion.java:8-10          enum {LOSSY, LOSSLESS}
 *           -> JP2HIP_LOSSY = 0, JP2HIP_LOSSLESS = 1 (same ordinals).
 *   converters/KakaduConverter.java:38-44    BASE_OPTIONS + LOSSLESS_OPTIONS /
 *                                            LOSSY_OPTION (the kdu recipe)
 *           -> jp2hip_recipe / jp2hip_recipe_init().
 *   converters/KakaduConverter.java:61-71    fork/exec of kdu_compress
 *           -> in-process call; no child process.
 *   converters/ConverterFactory.java:86-103  checkSystemKakadu() probe
 *           -> jp2hip_probe() (a device with gfx950 is visible).
 *
 * All pointers are plain host pointers unless the name says d_ (device).
 * Paths are UTF-8 bytes.  Calls on one context are serialised internally;
 * different contexts (one per GPU) run concurrently.
 */
#ifndef JP2HIP_H
#define JP2HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define JP2HIP_LOSSY 0    /* Conversion.LOSSY    (Conversion.java:9)  */
#define JP2HIP_LOSSLESS 1 /* Conversion.LOSSLESS (Conversion.java:9)  */

#define JP2HIP_FORMAT_J2K 0 /* raw codestream                          */
#define JP2HIP_FORMAT_JP2 1
#define JP2HIP_FORMAT_JPX 2 /* what a ".jpx" output name asks Kakadu for */

typedef struct jp2hip_ctx jp2hip_ctx;

typedef struct jp2hip_config {
    int32_t device;       /* HIP device ordinal                                */
    int32_t host_threads; /* tier-2 worker threads (<=0: min(16, hw threads))  */
    int32_t profile;      /* 1: record per-stage HIP event times in stats      */
    int32_t reserved;
} jp2hip_config;

/* The kdu_compress recipe (KakaduConverter.java:38-44), field by field. */
typedef struct jp2hip_recipe {
    int32_t levels;          /* Clevels=6                                      */
    int32_t layers;          /* Clayers=6                                      */
    int32_t tile_w, tile_h;  /* Stiles={512,512}                               */
    int32_t cblk_w_log2;     /* Cblk={64,64}                                   */
    int32_t cblk_h_log2;
    int32_t nprecincts;      /* Cprecincts={256,256},{256,256},{128,128}:     */
    int32_t prec_w_log2[16]; /*   highest resolution first, last one repeats   */
    int32_t prec_h_log2[16];
    int32_t progression;     /* Corder=RPCL (2); the only order implemented    */
    int32_t sop, eph;        /* Cuse_sop=yes Cuse_eph=yes                      */
    int32_t plt;             /* ORGgen_plt=yes                                 */
    int32_t tparts_r;        /* ORGtparts=R                                    */
    int32_t guard_bits;      /* 1                                              */
    int32_t reversible;      /* Creversible=yes -> 5/3 + RCT, else 9/7 + ICT   */
    int32_t mct;             /* colour transform on components 0..2            */
    double qstep;            /* irreversible base step (Kakadu Qstep=1/256)    */
    double rate_bpp;         /* "-rate 3"; <= 0 means "-rate -" (all passes)   */
    int32_t format;          /* JP2HIP_FORMAT_*                                */
    int32_t comment;         /* emit Kakadu-style COM markers: a version       */
                             /* string and "Kdu-Layer-Info" (layer slopes and  */
                             /* bytes, test.jpx's second COM)                  */
    int32_t slope_skip;      /* rate-driven (rate_bpp > 0) only: do not code   */
                             /* bit-planes whose predicted slope lies far      */
                             /* below the rate target's, as kdu_compress's     */
                             /* block coder does under "-rate"; 0 = code all   */
    int32_t flush_period;    /* -flush_period 1024 (KakaduConverter.java:40):  */
                             /* tile-parts go out per stripe of tile rows that */
                             /* completes a flush -- resolution 0 of every     */
                             /* tile in the stripe, then resolution 1, ...     */
                             /* (test.jpx's order); <= 0: tile after tile      */
} jp2hip_recipe;

/* Where the samples live inside a source buffer (a baseline TIFF's strips). */
typedef struct jp2hip_layout {
    int32_t width, height, components, bits; /* bits 8 or 16, unsigned      */
    int32_t planar;                          /* 1 chunky, 2 planar          */
    int32_t big_endian;                      /* 16-bit sample byte order    */
    int32_t rows_per_strip;
    int32_t nstrips;                         /* entries in strip_offsets    */
    const uint64_t *strip_offsets;           /* byte offset of each strip   */
    int32_t compression;                     /* TIFF Compression: 1 (or 0)  */
                                             /* none, 5 LZW, 8 / 32946      */
                                             /* Deflate, 32773 PackBits     */
    int32_t predictor;                       /* TIFF Predictor: 1 none,     */
                                             /* 2 horizontal differencing   */
    const uint64_t *strip_bytes;             /* compressed size per strip   */
                                             /* (compression > 1)           */
    int32_t tile_width, tile_height;         /* tiled TIFF (0: strips): the */
                                             /* "strips" above are then the */
                                             /* tiles, row-major per plane  */
} jp2hip_layout;

/* Stage times (ingest_ms .. t2_ms, t1_cm_ms, t1_mq_ms) come from HIP events
 * and are filled only for a context created with jp2hip_config.profile = 1
 * (0 otherwise); total_ms, h2d_ms and the counts are always filled. */
typedef struct jp2hip_stats {
    double total_ms;      /* host wall time of the call                       */
    double h2d_ms;        /* source upload (encode_file / encode_tiff only)   */
    double ingest_ms;     /* strip gather + level shift + RCT/ICT kernel      */
    double dwt_ms;        /* all DWT kernels                                  */
    double quant_ms;      /* quantisation + bit-plane kernel                  */
    double t1_ms;         /* EBCOT tier-1 kernels                             */
    double pcrd_ms;       /* hull + threshold selection kernels               */
    double d2h_ms;        /* metadata + compressed bytes download             */
    double t2_ms;         /* tier-2 on the device: packet headers, tile-part  */
                          /* sizing and code-stream emission                  */
    int64_t codeblocks;
    int64_t coded_passes;
    int64_t t1_bytes;     /* MQ bytes produced by tier-1 (before truncation)  */
    int64_t out_bytes;
    int32_t rate_iterations;
    int32_t host_waits;   /* times the host blocked on the GPU during the encode */
    double t1_cm_ms;      /* tier-1 context-modelling kernel (part of t1_ms)  */
    double t1_mq_ms;      /* tier-1 MQ-coder kernel (part of t1_ms)           */
    int64_t mq_decisions; /* MQ-coded decisions (one decision-stream byte each) */
    int64_t stream_pool_bytes; /* tier-1 decision-stream pool held by the context */
    int64_t stream_need_bytes; /* ... of which this encode's coded planes took    */
    int32_t pool_grows;   /* encodes repeated because the pool was short (0..2) */
    int32_t reserved;
} jp2hip_stats;

const char *jp2hip_version(void);

/* Thread-local message for the last failing call on this thread. */
const char *jp2hip_last_error(void);

/* 1 if a gfx950 device is usable (ConverterFactory.checkSystemKakadu analogue). */
int jp2hip_probe(void);

/* Number of visible HIP devices that are gfx950 (0 if none). */
int jp2hip_device_count(void);

/* The HIP ordinals of the visible gfx950 devices (what jp2hip_config.device
 * takes), at most `max` of them written to `ordinals`; returns how many there
 * are.  A converter spreads its contexts over these, not over 0..n-1 (a
 * non-gfx950 device may hold a low ordinal). */
int jp2hip_device_ordinals(int32_t *ordinals, int32_t max);

/* "" when the process environment suits the contexts alive in it, else
 * what to change: GPU_MAX_HW_QUEUES below the live context count (contexts
 * sharing a hardware queue run their kernels one after another).  It must
 * be set before the library loads; a converter logs this once after
 * creating its contexts. */
const char *jp2hip_env_check(void);

/* Fill the Bucketeer recipe for JP2HIP_LOSSY / JP2HIP_LOSSLESS. */
void jp2hip_recipe_init(jp2hip_recipe *recipe, int conversion);

int jp2hip_create(jp2hip_ctx **out, const jp2hip_config *cfg);
void jp2hip_destroy(jp2hip_ctx *ctx);

/* Device memory (bytes) held by a context's buffers, its tile-split members'
 * included.  Buffers grow to what the largest recent image needed. */
int64_t jp2hip_device_bytes(jp2hip_ctx *ctx);

/* A context's device-memory policy, its tile-split members' too.
 * soft: bytes it may keep between encodes; an encode that leaves it above
 *   releases every buffer at its end (<= 0, the default: relative to the
 *   context's usual image -- it releases when it holds more than twice the
 *   larger of the median of what its last 8 encodes needed and what the
 *   encode before this one needed, plus 256 MiB, so one outsized master
 *   does not pin HBM for the context's life, a steady run of large masters
 *   keeps its buffers, and a lasting change to larger images costs one
 *   release).
 * hard: bytes no encode may pass; an image that needs more fails with
 *   rc < 0 and a message (never a fault), and the context stays usable
 *   (<= 0: no limit but the device's).
 * When the device itself runs out of memory, the allocating encode takes
 * back the buffers of idle contexts of the same device and waits (up to
 * 30 s) for busy ones to become idle before it fails.
 * Returns 0, or < 0 for a null context. */
int jp2hip_set_memory_limits(jp2hip_ctx *ctx, int64_t soft, int64_t hard);

/* Which SDMA engines the code-stream copies use, per GPU probed so far, and
 * every engine's measured device -> host rate ("" before the first encode):
 * engines differ several-fold on MI355X and the choice is timed once per
 * GPU, so a benchmark records it to be comparable with another run. */
const char *jp2hip_dma_engines(void);

/* Free and total memory of HIP device `device` (bytes): what a converter
 * sizes its context pool from.  Returns 0 or < 0. */
int jp2hip_device_memory(int device, int64_t *free_bytes, int64_t *total_bytes);

/* Converter.convert(): TIFF file -> JPEG 2000 file, written atomically
 * (temp file + rename; nothing is left behind on failure).
 * recipe == NULL -> jp2hip_recipe_init(conversion).  Returns 0 or < 0. */
int jp2hip_encode_file(jp2hip_ctx *ctx, const char *tiff_path_utf8, const char *out_path_utf8,
                       int conversion, const jp2hip_recipe *recipe, jp2hip_stats *stats);

/* TIFF bytes in host memory -> encoded bytes.  *out is pinned host memory
 * (the code-stream is copied straight into it from HBM); release it with
 * jp2hip_free, never free(). */
int jp2hip_encode_tiff(jp2hip_ctx *ctx, const uint8_t *tiff, size_t len, int conversion,
                       const jp2hip_recipe *recipe, uint8_t **out, size_t *out_len,
                       jp2hip_stats *stats);

/* Parse a baseline TIFF's header into a layout (offsets into the file).
 * Strips may be uncompressed, LZW (5), Deflate (8, 32946; zlib streams) or
 * PackBits (32773), with or without
 * horizontal differencing (Predictor 2); compressed strips are decoded on
 * the GPU before ingest (LZW segment-parallel: a wave finds a strip's
 * Clear-code segments, a wave per segment resolves its codes; Deflate and
 * PackBits a wave per strip).  For a compressed file
 * `offsets` receives 2 * nstrips entries: the strip offsets, then their byte
 * counts (layout->strip_bytes points at the second half).  Tiled TIFFs
 * (TileWidth/TileLength) are described the same way, one entry per tile,
 * and always carry the byte counts; they are untiled in HBM before ingest. */
int jp2hip_tiff_layout(const uint8_t *tiff, size_t len, jp2hip_layout *layout,
                       uint64_t *offsets, int32_t max_offsets);

/* Device-resident source: d_src holds the TIFF file (or any buffer the
 * layout describes) in HBM.  This is the entry the benchmark times. */
int jp2hip_encode_device(jp2hip_ctx *ctx, const void *d_src, size_t src_len,
                         const jp2hip_layout *layout, int conversion,
                         const jp2hip_recipe *recipe, uint8_t **out, size_t *out_len,
                         jp2hip_stats *stats);

/* Releases an *out buffer of the encode calls.  It returns to the process's
 * pool of pinned buffers, so steady-state encodes pin nothing new; the pool
 * keeps as many returned buffers as were ever handed out at once (each
 * counted at the largest size pinned), at least 4 GiB, and unpins the
 * largest beyond that. */
void jp2hip_free(void *p);

/* ------------------------------------------------------------------------
 * Tile-split path: one oversized image across GPUs.
 *
 * No reference interface exists for this (kdu_compress encodes one image in
 * one process, KakaduConverter.java:61-71); it is the north_star's "RCCL only
 * if a single oversized image is split across GPUs".  Rank r of `world`
 * encodes the contiguous band of tile rows jp2hip_split_rows() names
 * (ingest, DWT, tier-1 and hulls of its tiles only); the ranks agree on the
 * PCRD layer thresholds exactly through `allreduce_sum` (a caller-supplied
 * in-place int64 sum over ranks -- RCCL/torch.distributed on the node), so
 * the concatenation of every rank's part, in rank order, is byte-identical
 * to the single-GPU jp2hip_encode_device() output.  The only exchange is a
 * few hundred all-reduces of <= 64 int64 (threshold bisection, tier-2 sizes);
 * no pixel or coefficient crosses GPUs.
 * ---------------------------------------------------------------------- */
typedef int (*jp2hip_allreduce_fn)(void *user, int64_t *values, int32_t n); /* in-place sum; 0 ok */

typedef struct jp2hip_split {
    int32_t rank, world;
    jp2hip_allreduce_fn allreduce_sum; /* may be NULL when world == 1 */
    void *user;
} jp2hip_split;

/* Image rows [*row0, *row1) whose tiles rank `rank` encodes: whole
 * -flush_period stripes of tile rows (recipe.flush_period), so every rank's
 * tile-parts are one contiguous run of the file. */
void jp2hip_split_rows(int32_t height, int32_t tile_h, int32_t flush_period, int32_t rank, int32_t world,
                       int32_t *row0, int32_t *row1);

/* This rank's part of the file: *out (jp2hip_free) goes at byte *file_offset
 * of a *file_len-byte file.  Rank 0's part starts with the file and main
 * headers, the last rank's ends with EOC.  d_src/layout describe the whole
 * TIFF, but only the strips of this rank's rows are read, so d_src may hold
 * just those (with strip offsets relative to it).  Collective: every rank
 * must call it with the same image geometry and recipe. */
int jp2hip_encode_device_split(jp2hip_ctx *ctx, const void *d_src, size_t src_len,
                               const jp2hip_layout *layout, int conversion,
                               const jp2hip_recipe *recipe, const jp2hip_split *split,
                               uint8_t **out, size_t *out_len, uint64_t *file_offset,
                               uint64_t *file_len, jp2hip_stats *stats);

/* The tile-split behind Converter.convert (Converter.java:22 ->
 * jp2hip_encode_file / jp2hip_encode_tiff on ctx): gives ctx `n` peer
 * contexts, one on each HIP ordinal in `ordinals` (created here, owned by ctx;
 * an ordinal may repeat, or be ctx's own device).  From then on an image of at
 * least `min_pixels` pixels (width x height) given to ctx is encoded as a
 * tile-split over world = n + 1 ranks -- ctx is rank 0, peer i rank i + 1 --
 * each rank a thread of this call: it reads its band's strips from the TIFF
 * (mapped, not read whole), uploads them to its own GPU, and writes its part
 * at its offset of the output file; the ranks' exchanges are summed on the
 * host (no caller callback, no RCCL needed in-process).  The file is
 * byte-identical to the single-GPU encode.  Smaller images take the
 * single-GPU path.  n = 0 removes the peers.  Not to be called while ctx is
 * encoding.  Returns 0 or < 0. */
int jp2hip_split_peers(jp2hip_ctx *ctx, const int32_t *ordinals, int32_t n, int64_t min_pixels);

/* Width x height of a TIFF file from its header (the file is mapped, not
 * read), or < 0 with jp2hip_last_error(): lets a converter route an
 * oversized image to its split context before converting it. */
int64_t jp2hip_tiff_pixels(const char *tiff_path_utf8);

/* Host-only: global layer thresholds from this rank's hull segments (slope
 * keys descending, inclusive byte sums) -- the exchange step of the split
 * encode, exported for tests.  K[l] = min{k : sum over ranks of bytes with
 * key >= k <= budgets[l]}. */
int jp2hip_split_thresholds(const uint64_t *keys, const int64_t *cum, int64_t nseg,
                            const int64_t *budgets, int32_t layers, const jp2hip_split *split,
                            uint64_t *K);

/* ------------------------------------------------------------------------
 * Batch path: one GPU's work queue for a CSV batch.
 *
 * Replaces the chain a CSV row takes through the reference
 *   LoadCsvHandler.java:250-289 -> LargeImageVerticle.java:65-108 ->
 *   ImageWorkerVerticle.java:54-110 (convert LOSSLESS, reply, then hand the
 *   JPX to S3BucketVerticle with derivative-image=true) ->
 *   S3BucketVerticle.java:88-211,286-303 (PUT, delete the JPX after a
 *   successful upload)
 * with a native pipeline per GPU: reader threads (TIFF file -> pinned host
 * buffer, header parse), one encoder thread per context (images in flight on
 * the GPU, each with its own HIP stream), and uploader threads (atomic JPX
 * write, upload callback, delete-after-upload), so file I/O and the upload
 * overlap the encodes.  Images are independent: N GPUs run N of these
 * (one process per GPU), sharded by the caller; no collective.
 * ---------------------------------------------------------------------- */
typedef struct jp2hip_batch jp2hip_batch;

/* Upload hook (S3BucketVerticle stand-in): called on an uploader thread with
 * the image id (S3 key = file name, ImageWorkerVerticle.java:69) and the
 * written JPX path.  Return 0 on success.  NULL selects the built-in stub,
 * which reads every byte of the file and succeeds (FakeS3BucketVerticle). */
typedef int (*jp2hip_upload_fn)(void *user, const char *image_id_utf8, const char *jpx_path_utf8);

typedef struct jp2hip_batch_config {
    int32_t device;              /* HIP device ordinal                               */
    int32_t contexts;            /* images in flight on the GPU (<=0: 12)            */
    int32_t reader_threads;      /* TIFF readers (<=0: 4)                            */
    int32_t uploader_threads;    /* JPX writers + uploaders (<=0: 4)                 */
    int32_t host_threads;        /* tier-2 threads per context (<=0: 16 / contexts)  */
    int32_t delete_after_upload; /* derivative-image=true: remove the JPX once sent  */
    int32_t write_output;        /* 0: keep the JPX in memory, skip the file write   */
    int32_t reserved;
} jp2hip_batch_config;

#define JP2HIP_BATCH_OK 0
#define JP2HIP_BATCH_CONVERT_FAILED (-1) /* ImageWorker replies failure (IOException) */
#define JP2HIP_BATCH_UPLOAD_FAILED (-2)  /* S3 upload failed; callback gets "false"   */

typedef struct jp2hip_batch_result {
    int64_t job;          /* the caller's job number from jp2hip_batch_submit     */
    int32_t status;       /* JP2HIP_BATCH_*                                       */
    int32_t reserved;
    int64_t in_bytes;     /* TIFF file size                                       */
    int64_t out_bytes;    /* JPX size                                             */
    int64_t pixels;       /* width * height                                       */
    double read_ms;       /* file -> pinned buffer + header parse                 */
    double encode_ms;     /* H2D + GPU encode + tier-2 (jp2hip_encode_tiff)       */
    double upload_ms;     /* file write + upload hook + delete                    */
    char message[240];    /* failure text ("" on success)                         */
} jp2hip_batch_result;

int jp2hip_batch_create(jp2hip_batch **out, const jp2hip_batch_config *cfg, jp2hip_upload_fn upload,
                        void *user);
/* Queue one image: convert `tiff_path` into `jpx_path` (written atomically)
 * with `conversion` (recipe NULL -> Bucketeer recipe), then upload it under
 * `image_id`.  Never blocks on the GPU; returns < 0 after close. */
int jp2hip_batch_submit(jp2hip_batch *b, int64_t job, const char *image_id_utf8, const char *tiff_path_utf8,
                        const char *jpx_path_utf8, int conversion, const jp2hip_recipe *recipe);
/* Collect up to `max` finished jobs (uploaded or failed); waits up to
 * timeout_ms (< 0: until at least one is ready or nothing is pending).
 * Returns the number written to `results`. */
int jp2hip_batch_wait(jp2hip_batch *b, jp2hip_batch_result *results, int max, int timeout_ms);
/* Jobs submitted and not yet returned by jp2hip_batch_wait. */
int64_t jp2hip_batch_pending(jp2hip_batch *b);
/* Stop accepting jobs, finish the queued ones, join all threads. */
void jp2hip_batch_destroy(jp2hip_batch *b);

#ifdef __cplusplus
}
#endif
#endif
