// Host build of k_inflate (kernels.hip), for the CPU test suite: the kernel's
// text is spliced in by tests/test_inflate_host.py between this file's shims
// and main(), compiled with clang++ -fsanitize=address, and run on zlib
// streams (levels 0/1/6/9 at every byte alignment) and damaged streams.
// [[SHIMS]]
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>
#include <algorithm>
#include <zlib.h>
#define __device__
#define __host__
#define __forceinline__ inline
#define __global__
#define __launch_bounds__(x)
#define __shared__ static
#define __constant__ static const
#define JP2HIP_INF_LANES 1
#define __builtin_amdgcn_readfirstlane(x) (x)
#define __builtin_amdgcn_wave_barrier() ((void)0)
#define __builtin_amdgcn_readlane(v, l) (v)  /* one lane: the only lane is 0 */
#define __popcll(x) __builtin_popcountll(x)
static inline uint32_t __builtin_amdgcn_alignbit(uint32_t hi, uint32_t lo, uint32_t s) {
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> (s & 31));
}
struct uint4 { uint32_t x, y, z, w; };
static inline uint4 make_uint4(uint32_t x, uint32_t y, uint32_t z, uint32_t w) { return uint4{x, y, z, w}; }
static struct { int x, y; } blockIdx, threadIdx;
static inline int atomicOr(int *p, int v) { int o = *p; *p |= v; return o; }
static inline uint32_t atomicAdd(uint32_t *p, uint32_t v) { uint32_t o = *p; *p += v; return o; }
using std::min;
// [[MAIN]]
using namespace jp2hip;

// lnk_init: what the link buffer holds before the decode (a fresh context's
// hipMalloc memory may hold zeros, a reused one stale links of another image)
static int run(const std::vector<uint8_t> &z, int off, const std::vector<uint8_t> &raw,
               uint32_t lnk_init = 0xDEADBEEFu) {
    std::vector<uint8_t> buf(z.size() + 16, 0xA5);
    std::memcpy(buf.data() + off, z.data(), z.size());
    std::vector<uint8_t> out(raw.size() + 256);
    std::vector<uint32_t> lnk(raw.size() + 256, lnk_init);
    uint64_t o = off, c = z.size();
    int err = 0;
    UnpackArgs a{};
    a.src = buf.data(); a.off = &o; a.cnt = &c; a.nstrips = 1;
    a.unit_bytes = raw.size(); a.stride = raw.size() + 256; a.dst = out.data(); a.err = &err;
    a.lnk = lnk.data();
    blockIdx.x = 0; blockIdx.y = 0; threadIdx.x = 0;
    k_inflate(a);
    // k_inflate_links as the GPU runs it (also after a failed decode: it is
    // launched unconditionally, so it must end in bounds on any link
    // contents): doubling rounds, then the chase
    const int chunks = (int)((raw.size() + kLinkChunk - 1) / kLinkChunk);
    for (int r = 0; r <= kLinkDoublings; r++)
        for (int bx = 0; bx < chunks; bx++)
            for (int t = 0; t < 256; t++) {
                blockIdx.x = bx; threadIdx.x = t;
                k_inflate_links(a, r == kLinkDoublings ? 1 : 0);
            }
    blockIdx.x = 0; threadIdx.x = 0;
    if (err) return 1;
    return std::memcmp(out.data(), raw.data(), raw.size()) ? 2 : 0;
}

int main() {
    std::vector<uint8_t> raw(300000);
    uint32_t r = 1;
    for (size_t i = 0; i < raw.size(); i++) {
        r = r * 1103515245u + 12345u;
        raw[i] = (uint8_t)((i / 7) % 50 + ((r >> 16) & 7));
    }
    int fails = 0;
    for (int lvl : {0, 1, 6, 9}) {
        uLongf cl = compressBound(raw.size());
        std::vector<uint8_t> z(cl);
        compress2(z.data(), &cl, raw.data(), raw.size(), lvl);
        z.resize(cl);
        for (int off = 0; off < 4; off++) {
            const int rc = run(z, off, raw);
            printf("level %d offset %d -> %d\n", lvl, off, rc);
            fails += rc != 0;
        }
        std::vector<uint8_t> t(z.begin(), z.begin() + z.size() / 2);  // truncated: must fail
        const int rt = run(t, 1, raw);
        printf("level %d truncated -> %d\n", lvl, rt);
        fails += rt != 1;
        // the same with a zeroed / self-referencing link buffer (ADVICE r4:
        // a zero link used to chase L[0] = 0 forever)
        for (uint32_t init : {0u, 5u, 0x7FFFFFFFu}) {
            const int rz = run(t, 1, raw, init);
            printf("level %d truncated, links preset %u -> %d\n", lvl, init, rz);
            fails += rz != 1;
        }
    }
    uLongf cl = compressBound(raw.size());
    std::vector<uint8_t> z(cl);
    compress2(z.data(), &cl, raw.data(), raw.size(), 6);
    z.resize(cl);
    z[2] = 0x07;  // BFINAL 1, BTYPE 3 (reserved)
    const int rb = run(z, 0, raw);
    printf("reserved block -> %d\n", rb);
    fails += rb != 1;
    const int rb0 = run(z, 0, raw, 0u);
    printf("reserved block, links preset 0 -> %d\n", rb0);
    fails += rb0 != 1;
    // long runs: chains of matches of matches (the links' doubling + chase),
    // and the strip ending inside a match / inside a stored block (a decoded
    // stream longer than the strip is cut, as libtiff does)
    std::vector<uint8_t> flat(700000, 0);
    for (size_t i = 0; i < flat.size(); i++) flat[i] = (uint8_t)(i < 1000 ? i * 7 : (i < 400000 ? 3 : (i / 5000) & 1));
    for (int lvl : {0, 1, 9}) {
        uLongf fl = compressBound(flat.size());
        std::vector<uint8_t> zf(fl);
        compress2(zf.data(), &fl, flat.data(), flat.size(), lvl);
        zf.resize(fl);
        const int rf = run(zf, 2, flat);
        printf("flat level %d -> %d\n", lvl, rf);
        fails += rf != 0;
        std::vector<uint8_t> cut(flat.begin(), flat.begin() + 654321);
        const int rc = run(zf, 3, cut);
        printf("flat level %d, strip shorter than the stream -> %d\n", lvl, rc);
        fails += rc != 0;
    }
    printf("%s\n", fails ? "FAIL" : "OK");
    return fails ? 1 : 0;
}
