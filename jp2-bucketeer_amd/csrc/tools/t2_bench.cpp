// Host-only timing harness for tier-2 (no GPU): C2 geometry, synthetic layer tables.
#include <chrono>
#include <cstdio>
#include <random>
#include <cstring>
#include "../jp2hip_internal.h"
using namespace jp2hip;
int main(int argc, char **argv) {
    jp2hip_recipe rc;
    std::memset(&rc, 0, sizeof rc);
    rc.levels = 6; rc.layers = 6; rc.tile_w = rc.tile_h = 512; rc.cblk_w_log2 = rc.cblk_h_log2 = 6;
    rc.nprecincts = 3; rc.prec_w_log2[0] = rc.prec_h_log2[0] = 8; rc.prec_w_log2[1] = rc.prec_h_log2[1] = 8;
    rc.prec_w_log2[2] = rc.prec_h_log2[2] = 7; rc.progression = 2; rc.sop = rc.eph = rc.plt = rc.tparts_r = 1;
    rc.guard_bits = 1; rc.mct = 1; rc.qstep = 1.0 / 256; rc.rate_bpp = 3; rc.format = 2; rc.comment = 1;
    Plan plan; std::string err;
    if (!build_plan(plan, rc, 6000, 4000, 3, 8, err)) { printf("%s\n", err.c_str()); return 1; }
    int nb = plan.blocks.size(), L = 6;
    std::vector<uint8_t> P(nb), nl((size_t)nb * L); std::vector<int32_t> lr((size_t)nb * L);
    std::mt19937 rng(1);
    uint64_t tot = 0; std::vector<uint64_t> off(nb);
    for (int b = 0; b < nb; b++) {
        P[b] = 3 + rng() % 6; int np = 3 * P[b] - 2; int n = 0, r = 0;
        for (int l = 0; l < L; l++) { n = std::min(np, n + (int)(rng() % 4)); r += (n ? 60 + rng() % 200 : 0); nl[b * L + l] = n; lr[b * L + l] = n ? r : 0; }
        off[b] = tot; tot += lr[b * L + L - 1];
    }
    std::vector<uint8_t> data(tot + 16, 0x55);
    int threads = argc > 1 ? atoi(argv[1]) : 16;
    T2Input in{&plan, P.data(), nl.data(), lr.data(), nullptr, off.data(), threads};
    T2State st;
    std::vector<uint8_t> file;
    for (int rep = 0; rep < 5; rep++) {
        auto t0 = std::chrono::steady_clock::now();
        int64_t sz = t2_headers(in, st);
        auto t1 = std::chrono::steady_clock::now();
        in.data = data.data();
        size_t fh = file_header_bytes(plan);
        file.resize(fh + (size_t)sz);
        write_file_header(plan, (uint64_t)sz, file.data());
        t2_emit(in, st, file.data() + fh);
        auto t2 = std::chrono::steady_clock::now();
        printf("threads %d: header pass %.2f ms (%lld B), emit %.2f ms (%zu B)\n", threads,
               std::chrono::duration<double, std::milli>(t1 - t0).count(), (long long)sz,
               std::chrono::duration<double, std::milli>(t2 - t1).count(), file.size());
    }
    if (argc > 2) { FILE *fo = fopen(argv[2], "wb"); fwrite(file.data(), 1, file.size(), fo); fclose(fo); }
}
