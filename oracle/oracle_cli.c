/* oracle_cli.c -- TEST INFRASTRUCTURE ONLY: encode a TIFF with the oracle.
 * usage: oracle_cli in.tif out.(j2k|jp2|jpx) lossless|lossy [rate_bpp] */
#include "jp2_oracle.h"
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int main(int argc, char **argv) {
    if (argc < 4) { fprintf(stderr, "usage: %s in.tif out lossless|lossy [rate]\n", argv[0]); return 2; }
    FILE *f = fopen(argv[1], "rb");
    if (!f) { perror(argv[1]); return 1; }
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    unsigned char *buf = malloc((size_t)n);
    if (fread(buf, 1, (size_t)n, f) != (size_t)n) { fclose(f); return 1; }
    fclose(f);
    oracle_recipe r;
    oracle_recipe_init(&r, strcmp(argv[3], "lossless") == 0);
    if (argc > 4) r.rate_bpp = atof(argv[4]);
    const char *ext = strrchr(argv[2], '.');
    r.format = (ext && strcmp(ext, ".j2k") == 0) ? 0 : (ext && strcmp(ext, ".jp2") == 0 ? 1 : 2);
    unsigned char *out;
    size_t olen;
    if (oracle_encode_tiff(buf, (size_t)n, &r, &out, &olen)) { fprintf(stderr, "error: %s\n", oracle_last_error()); return 1; }
    f = fopen(argv[2], "wb");
    fwrite(out, 1, olen, f);
    fclose(f);
    printf("%zu\n", olen);
    return 0;
}
