/*
 * jp2_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the JPEG 2000 encode that Bucketeer's KakaduConverter
 * drives (`kdu_compress` with BASE_OPTIONS + LOSSLESS_OPTIONS / LOSSY_OPTION,
 * reference src/main/java/edu/ucla/library/bucketeer/converters/
 * KakaduConverter.java:38-44).  Kakadu itself is proprietary and absent, so
 * this is a restatement of ISO/IEC 15444-1 under that recipe (SURVEY.md
 * Appendix A).  It is pinned by the reference's only golden artifact,
 * src/test/resources/images/test.jpx (main-header bytes, packet/tile-part
 * structure, decoded pixels) and by opj_decompress round trips; see
 * tests/golden/make_golden.py.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library.  The product (libjp2hip) never links or calls it.
 */
#ifndef JP2_ORACLE_H
#define JP2_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Same field meaning as jp2hip_recipe in include/jp2hip.h (declared
 * separately on purpose: the oracle shares no code with the product). */
typedef struct oracle_recipe {
    int32_t levels;            /* Clevels=6                                  */
    int32_t layers;            /* Clayers=6                                  */
    int32_t tile_w, tile_h;    /* Stiles={512,512}                           */
    int32_t cblk_w_log2;       /* Cblk={64,64}                               */
    int32_t cblk_h_log2;
    int32_t nprecincts;        /* entries in prec_*; Kakadu order: highest   */
    int32_t prec_w_log2[16];   /* resolution first, last entry repeats       */
    int32_t prec_h_log2[16];   /* (Cprecincts={256,256},{256,256},{128,128}) */
    int32_t progression;       /* 2 = RPCL (Corder=RPCL), the only one       */
    int32_t sop, eph;          /* Cuse_sop=yes, Cuse_eph=yes                 */
    int32_t plt;               /* ORGgen_plt=yes                             */
    int32_t tparts_r;          /* ORGtparts=R                                */
    int32_t guard_bits;        /* 1 (Kakadu default, test.jpx QCD)           */
    int32_t reversible;        /* 1: Creversible=yes (5/3 + RCT); 0: 9/7+ICT */
    int32_t mct;               /* 1: RCT/ICT on components 0..2              */
    double qstep;              /* Qstep for irreversible, 1/256              */
    double rate_bpp;           /* -rate 3 ; <= 0 => "-rate -" (all passes)   */
    int32_t format;            /* 0 raw J2K codestream, 1 JP2, 2 JPX         */
    int32_t comment;           /* write a COM marker                         */
    int32_t slope_skip;        /* rate-driven only: skip bit-planes whose    */
                               /* predicted slope is far below the target's  */
                               /* (Kakadu-style slope prediction); 0 = off   */
    int32_t flush_period;      /* -flush_period 1024: tile-parts are written */
                               /* per stripe of tile rows that completes a   */
                               /* flush (res 0 of every tile in the stripe,  */
                               /* then res 1, ...); <= 0: tile by tile       */
} oracle_recipe;

/* Fill the Bucketeer recipe: lossless != 0 -> LOSSLESS_OPTIONS, else LOSSY. */
void oracle_recipe_init(oracle_recipe *r, int lossless);

/* Parse a baseline (uncompressed, strip) TIFF.  On success *pix points to a
 * malloc'd interleaved sample buffer (uint8, or host-endian uint16). */
int oracle_tiff_read(const uint8_t *buf, size_t len, int *w, int *h, int *nc,
                     int *bits, void **pix);

/* Encode interleaved samples.  *out is malloc'd (free with oracle_free). */
int oracle_encode(const void *pix, int w, int h, int nc, int bits,
                  const oracle_recipe *r, uint8_t **out, size_t *out_len);

/* TIFF bytes -> JPEG 2000 bytes (oracle_tiff_read + oracle_encode). */
int oracle_encode_tiff(const uint8_t *tiff, size_t len, const oracle_recipe *r,
                       uint8_t **out, size_t *out_len);

/* Stage probes used by the parity tests (tile-component level). */
/* Forward DWT of one tile-component in place (Mallat layout, stride = w).
 * reversible: data is int32; else float. */
void oracle_fdwt(void *data, int w, int h, int levels, int reversible);

/* T1-encode one code-block of sign-magnitude samples (bit 31 = sign).
 * band: 0 LL, 1 HL, 2 LH, 3 HH.  Returns number of passes; fills
 * out_bytes (capacity cap), *out_len, rates[npasses], dists[npasses]. */
int oracle_t1_encode(const int32_t *sm, int w, int h, int band, int lossless,
                     uint8_t *out_bytes, int cap, int *out_len,
                     int32_t *rates, int64_t *dists, int *nplanes);
/* Same, coding only bit-planes >= pmin (the planes slope prediction keeps). */
int oracle_t1_encode_planes(const int32_t *sm, int w, int h, int band, int lossless, int pmin,
                            uint8_t *out_bytes, int cap, int *out_len,
                            int32_t *rates, int64_t *dists, int *nplanes);

/* Debug: MQ decisions coded since the previous call (workload analysis). */
int64_t oracle_debug_decisions(void);

void oracle_free(void *p);
const char *oracle_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
