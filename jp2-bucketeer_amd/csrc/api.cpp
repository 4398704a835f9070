// api.cpp -- the C ABI of libjp2hip (include/jp2hip.h).
//
// jp2hip_encode_file() is the in-process replacement for the kdu_compress
// child process that KakaduConverter.convert() spawns
// (KakaduConverter.java:55-77 -> AbstractConverter.run, AbstractConverter.java:29-39):
// same inputs (TIFF path, output path, Conversion), same recipe, blocking,
// and every failure surfaces as a negative return code plus a message,
// never as a partially written output file.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstddef>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <unordered_map>
#include <thread>
#include <vector>

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include "gpu_encoder.h"
#include "jp2hip.h"
#include "jp2hip_internal.h"
#include "mem_policy.h"

// The last geometry's plan, tier-2 tables and main-header length: a batch of
// same-size images (the common case) builds them once (C2: ~5 ms of host
// time per encode otherwise), and the device keeps their tables resident.
struct PlanCache {
    bool valid = false;
    jp2hip_recipe rc;
    int w = 0, h = 0, nc = 0, bits = 0;
    jp2hip::Plan plan;
    jp2hip::T2Tables tabs;
    std::vector<uint8_t> mh0;
};

struct jp2hip_ctx {
    std::mutex mu;
    // whole tile-split encodes on this context, one at a time: each rank
    // takes its member's `mu`, so two concurrent splits could otherwise hold
    // one member each and wait for each other in an exchange
    std::mutex split_mu;
    jp2hip::GpuEncoder gpu;
    jp2hip_config cfg;
    int threads = 1;
    PlanCache pc;
    // tile-split members (jp2hip_split_peers): images of at least
    // split_min_pixels are encoded by this context (rank 0) and these
    // (ranks 1..), owned here
    std::vector<jp2hip_ctx *> peers;
    int64_t split_min_pixels = 0;
    // device memory policy (jp2hip_set_memory_limits): 0 = default
    int64_t mem_soft = 0;
    size_t dev_total = 0;  // the device's memory (hipMemGetInfo at create)
    std::vector<size_t> needs;  // what the last encodes asked for (the context's usual image)
    int64_t reclaimed = 0;      // times another context took this one's idle buffers
    ~jp2hip_ctx() {
        for (jp2hip_ctx *p : peers) jp2hip_destroy(p);
    }
};

namespace {

thread_local std::string g_err;

int fail(const std::string &msg) {
    g_err = msg;
    return -1;
}

// Every encode ends here, success or not: a failed one drains the stream
// first (no buffer is released while a kernel may still read it), then the
// context's device-memory policy decides whether it keeps its buffers.
//  - an explicit soft limit (jp2hip_set_memory_limits): release everything
//    when the context holds more;
//  - by default, relative to the context's usual image: release everything
//    when it holds more than twice the median of what its last 8 encodes
//    needed (plus 256 MiB) -- one C5-class master in a pool of C2 / C4 work
//    is released right after it, while a steady run of large masters (C3
//    every time) keeps its buffers instead of reallocating per image.
// Memory pressure between contexts is handled where it arises: an
// allocation that fails takes back what idle contexts of the device hold
// (reclaim_idle).
struct EncodeEnd {
    jp2hip_ctx *ctx;
    bool ok = false;
    ~EncodeEnd() {
        if (!ok) ctx->gpu.quiesce();
        if (ok) jp2hip::record_need(ctx->needs, ctx->gpu.need_bytes());
        const size_t limit = jp2hip::keep_limit(ctx->needs, ctx->mem_soft);  // (mem_policy.h)
        if (ctx->gpu.device_bytes() > limit) {
            ctx->gpu.quiesce();
            ctx->gpu.trim(limit);
        }
    }
};

// Contexts alive in this process (jp2hip_env_check, the pinned pool's cap).
static std::atomic<int> g_live_contexts{0};

// Encoded files are returned in pinned host memory: the final code-stream D2H
// lands in the caller's buffer directly (no staging copy; a C3 file is
// ~340 MB) and jp2hip_free() hands the buffer back to a pool, so steady state
// allocates and pins nothing.  The pool keeps returned buffers up to the
// most that were ever handed out at once, each counted at the largest size
// pinned so far (at least 4 GiB): with a fixed 4 GiB, twelve contexts of C3
// files (385 MB buffers) overflowed it whenever most of their files were
// returned at once, and the next encodes pinned fresh buffers --
// hipHostMalloc / hipHostFree of that size took tens of ms and held up the
// other contexts' launches meanwhile (a 19 ms window with no kernel on the
// GPU, profiles/r06/c3_pinned_pool.txt); a batch queue holds more files than
// contexts (its uploaders' queue), hence the high-water mark rather than the
// context count.  jp2hip_free() of a pointer the pool does not know is plain
// free().
struct PinnedPool {
    std::mutex mu;
    std::unordered_map<void *, size_t> live;   // handed out: capacity
    std::multimap<size_t, void *> idle;        // returned: capacity -> buffer
    size_t idle_bytes = 0;
    size_t max_cap = 0;                        // the largest buffer pinned so far
    size_t peak_live = 0;                      // the most buffers handed out at once
    static constexpr size_t kIdleFloor = (size_t)4 << 30;
    size_t idle_cap() const {
#ifdef JP2HIP_POOL_FIXED_CAP  // A/B: the fixed 4 GiB of rounds 2-5
        return kIdleFloor;
#endif
        return std::max(kIdleFloor, peak_live * max_cap);
    }
};
PinnedPool &pinned_pool() {
    static PinnedPool *p = new PinnedPool();  // never destroyed: buffers may be freed at exit
    return *p;
}

uint8_t *out_alloc(size_t n) {
    PinnedPool &P = pinned_pool();
    n = std::max<size_t>(n, 1);
    {
        std::lock_guard<std::mutex> lk(P.mu);
        auto it = P.idle.lower_bound(n);
        if (it != P.idle.end() && it->first <= 2 * n + ((size_t)1 << 20)) {
            void *b = it->second;
            P.live[b] = it->first;
            P.peak_live = std::max(P.peak_live, P.live.size());
            P.idle_bytes -= it->first;
            P.idle.erase(it);
            return (uint8_t *)b;
        }
    }
    const size_t cap = n + n / 8 + 4096;  // room for a slightly larger file next time
    void *b = nullptr;
    static const bool log = getenv("JP2HIP_LOG_POOL") != nullptr;  // diagnostics: pool misses
    const auto t0 = std::chrono::steady_clock::now();
    if (hipHostMalloc(&b, cap, hipHostMallocDefault) != hipSuccess || !b) return nullptr;
    if (log) {
        std::lock_guard<std::mutex> lk(P.mu);
        fprintf(stderr, "jp2hip pool miss: %zu bytes pinned in %.1f ms (idle %zu buffers, %zu bytes)\n", cap,
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(),
                P.idle.size(), P.idle_bytes);
    }
    std::lock_guard<std::mutex> lk(P.mu);
    P.live[b] = cap;
    P.peak_live = std::max(P.peak_live, P.live.size());
    P.max_cap = std::max(P.max_cap, cap);
    return (uint8_t *)b;
}

void out_free(void *p) {
    if (!p) return;
    PinnedPool &P = pinned_pool();
    std::vector<void *> drop;
    {
        std::lock_guard<std::mutex> lk(P.mu);
        auto it = P.live.find(p);
        if (it == P.live.end()) {
            std::free(p);
            return;
        }
        const size_t cap = it->second;
        P.live.erase(it);
        P.idle.emplace(cap, p);
        P.idle_bytes += cap;
        const size_t idle_cap = P.idle_cap();
        while (P.idle_bytes > idle_cap && !P.idle.empty()) {  // largest first
            auto last = std::prev(P.idle.end());
            P.idle_bytes -= last->first;
            drop.push_back(last->second);
            P.idle.erase(last);
        }
    }
    for (void *b : drop) (void)hipHostFree(b);
}

double now_ms() {
    using namespace std::chrono;
    return duration<double, std::milli>(steady_clock::now().time_since_epoch()).count();
}

// ---- baseline TIFF header parsing (tags 256-339; classic TIFF and BigTIFF) ----
struct TiffReader {
    const uint8_t *b;
    size_t n;
    bool le;
    bool big = false;  // BigTIFF: 8-byte offsets, 20-byte IFD entries
    uint64_t un(size_t o, int k) const {
        if (o + (size_t)k > n || o + (size_t)k < o) return 0;
        uint64_t v = 0;
        for (int i = 0; i < k; i++) v |= (uint64_t)b[o + (le ? i : k - 1 - i)] << (8 * i);
        return v;
    }
    uint32_t u16(size_t o) const { return (uint32_t)un(o, 2); }
    uint32_t u32(size_t o) const { return (uint32_t)un(o, 4); }
    uint64_t u64(size_t o) const { return un(o, 8); }
    size_t entry_size() const { return big ? 20 : 12; }
    uint64_t count(size_t e) const { return big ? u64(e + 4) : u32(e + 4); }
    // value i of the entry at e (SHORT, LONG, LONG8 or BYTE)
    uint64_t val(size_t e, uint64_t i) const {
        const uint32_t type = u16(e + 2);
        const uint64_t cnt = count(e);
        const uint32_t sz = type == 3 ? 2 : (type == 4 ? 4 : (type == 16 ? 8 : 1));
        const size_t inl = big ? 8 : 4, voff = big ? e + 12 : e + 8;
        const uint64_t base = (uint64_t)sz * cnt <= inl ? voff : (big ? u64(voff) : u32(voff));
        if (i >= cnt) return 0;
        const size_t at = (size_t)(base + (uint64_t)sz * i);
        return sz == 2 ? u16(at) : (sz == 4 ? u32(at) : (sz == 8 ? u64(at) : (at < n ? b[at] : 0)));
    }
};

int parse_tiff(const uint8_t *buf, size_t len, jp2hip_layout *lay, std::vector<uint64_t> &offs) {
    if (!buf || len < 8) return fail("tiff: input too short");
    TiffReader t{buf, len, true};
    if (buf[0] == 'I' && buf[1] == 'I') t.le = true;
    else if (buf[0] == 'M' && buf[1] == 'M') t.le = false;
    else return fail("tiff: bad byte-order mark");
    size_t ifd, ifd_hdr;
    if (t.u16(2) == 43) {  // BigTIFF: offset size 8, reserved 0, first IFD at 8
        if (t.u16(4) != 8 || t.u16(6) != 0 || len < 16) return fail("tiff: bad BigTIFF header");
        t.big = true;
        ifd = (size_t)t.u64(8);
        ifd_hdr = 8;
    } else if (t.u16(2) == 42) {
        ifd = t.u32(4);
        ifd_hdr = 2;
    } else {
        return fail("tiff: not a TIFF file");
    }
    if (ifd + ifd_hdr > len || ifd + ifd_hdr < ifd) return fail("tiff: IFD offset out of range");
    const uint64_t ne = t.big ? t.u64(ifd) : t.u16(ifd);
    uint32_t w = 0, h = 0, spp = 1, bps = 8, comp = 1, planar = 1, rps = 0xFFFFFFFFu, fmt = 1, pred = 1;
    uint32_t photo = 0xFFFFFFFFu;  // absent: inferred from SamplesPerPixel
    size_t e_off = 0, e_cnt = 0;
    uint32_t n_off = 0, tw = 0, th = 0;
    if (ne > (len - ifd - ifd_hdr) / t.entry_size()) return fail("tiff: truncated IFD");
    for (uint64_t i = 0; i < ne; i++) {
        size_t e = ifd + ifd_hdr + t.entry_size() * (size_t)i;
        switch (t.u16(e)) {
        case 256: w = (uint32_t)t.val(e, 0); break;
        case 257: h = (uint32_t)t.val(e, 0); break;
        case 258: bps = (uint32_t)t.val(e, 0); break;
        case 259: comp = (uint32_t)t.val(e, 0); break;
        case 262: photo = (uint32_t)t.val(e, 0); break;
        case 273: e_off = e; n_off = (uint32_t)std::min<uint64_t>(t.count(e), 0xFFFFFFFFu); break;
        case 277: spp = (uint32_t)t.val(e, 0); break;
        case 278: rps = (uint32_t)std::min<uint64_t>(t.val(e, 0), 0xFFFFFFFFu); break;
        case 279: e_cnt = e; break;
        case 284: planar = (uint32_t)t.val(e, 0); break;
        case 317: pred = (uint32_t)t.val(e, 0); break;
        case 322: tw = (uint32_t)t.val(e, 0); break;
        case 323: th = (uint32_t)t.val(e, 0); break;
        case 324: e_off = e; n_off = (uint32_t)std::min<uint64_t>(t.count(e), 0xFFFFFFFFu); break;  // TileOffsets
        case 325: e_cnt = e; break;                                                                  // TileByteCounts
        case 339: fmt = (uint32_t)t.val(e, 0); break;
        default: break;
        }
    }
    if (!w || !h || !e_off) return fail("tiff: missing ImageWidth/ImageLength/StripOffsets");
    const bool tiled = tw || th;
    if (tiled && (!tw || !th || (tw % 16) || (th % 16) || tw > 65536 || th > 65536))
        return fail("tiff: bad TileWidth/TileLength");
    if (tiled && !e_cnt) return fail("tiff: tiles need TileByteCounts");
    // strips: uncompressed, LZW, Deflate or PackBits (decoded on the GPU,
    // kernels.hip k_unlzw / k_inflate / k_unpackbits); JPEG / CCITT are not
    if (comp != 1 && comp != 5 && comp != 8 && comp != 32946 && comp != 32773)
        return fail("tiff: compression " + std::to_string(comp) +
                    " is not supported (uncompressed, LZW, Deflate and PackBits only)");
    if (pred != 1 && pred != 2) return fail("tiff: predictor " + std::to_string(pred) + " is not supported");
    if (pred == 2 && comp == 1) return fail("tiff: predictor 2 without compression is not supported");
    if (comp != 1 && !e_cnt) return fail("tiff: compressed strips need StripByteCounts");
    if (bps != 8 && bps != 16) return fail("tiff: " + std::to_string(bps) + " bits/sample is not supported");
    if (fmt != 1) return fail("tiff: only unsigned integer samples are supported");
    if (spp < 1 || spp > 4) return fail("tiff: " + std::to_string(spp) + " samples/pixel is not supported");
    if (planar != 1 && planar != 2) return fail("tiff: bad PlanarConfiguration");
    // PhotometricInterpretation: BlackIsZero gray (+ alpha) or RGB (+ alpha);
    // the colour transform assumes RGB in components 0..2
    if (photo == 0xFFFFFFFFu) photo = spp >= 3 ? 2 : 1;
    if (photo == 0) return fail("tiff: PhotometricInterpretation 0 (WhiteIsZero) is not supported");
    if (photo != 1 && photo != 2)
        return fail("tiff: PhotometricInterpretation " + std::to_string(photo) +
                    " is not supported (BlackIsZero gray or RGB only)");
    if (photo == 2 && spp < 3) return fail("tiff: RGB needs 3 or 4 samples/pixel");
    if (photo == 1 && spp > 2) return fail("tiff: BlackIsZero with more than 2 samples/pixel is not supported");
    if (rps == 0 && !tiled) rps = h;  // RowsPerStrip 0 is invalid; libtiff reads it as one strip
    if (rps > h) rps = h;
    if (tiled) rps = th;  // per-unit rows (tiles are never clipped)
    const uint32_t across = tiled ? (w + tw - 1) / tw : 1;
    uint32_t per_plane = tiled ? across * ((h + th - 1) / th) : (h + rps - 1) / rps;
    uint32_t need = per_plane * (planar == 2 ? spp : 1);
    if (n_off < need) return fail(tiled ? "tiff: too few tiles" : "tiff: too few strips");
    const bool packed = comp != 1 || tiled;
    offs.resize(packed ? 2 * (size_t)need : need);
    size_t row = (size_t)w * (planar == 2 ? 1 : spp) * (bps / 8);
    for (uint32_t s = 0; s < need; s++) {
        offs[s] = t.val(e_off, s);
        uint32_t y0 = (s % per_plane) * rps;
        uint32_t rows = std::min(rps, h - y0);
        if (packed) {
            const uint64_t nb = t.val(e_cnt, s);
            if (offs[s] > len || nb > len - offs[s]) return fail("tiff: strip " + std::to_string(s) + " out of range");
            const uint64_t unit = (uint64_t)tw * (planar == 2 ? 1 : spp) * (bps / 8) * th;
            if (tiled && comp == 1 && nb < unit) return fail("tiff: tile byte count too small");
            offs[need + s] = nb;
            continue;
        }
        if (offs[s] > len || (uint64_t)row * rows > len - offs[s])
            return fail("tiff: strip " + std::to_string(s) + " out of range");
        if (e_cnt && t.val(e_cnt, s) < row * rows) return fail("tiff: strip byte count too small");
    }
    lay->width = (int32_t)w;
    lay->height = (int32_t)h;
    lay->components = (int32_t)spp;
    lay->bits = (int32_t)bps;
    lay->planar = (int32_t)planar;
    lay->big_endian = t.le ? 0 : 1;
    lay->rows_per_strip = (int32_t)rps;
    lay->nstrips = (int32_t)need;
    lay->strip_offsets = offs.data();
    lay->compression = (int32_t)comp;
    lay->predictor = (int32_t)pred;
    lay->strip_bytes = packed ? offs.data() + need : nullptr;
    lay->tile_width = (int32_t)tw;
    lay->tile_height = (int32_t)th;
    return 0;
}

void default_recipe(jp2hip_recipe *r, int conversion) {
    std::memset(r, 0, sizeof *r);
    r->levels = 6;
    r->layers = 6;
    r->tile_w = r->tile_h = 512;
    r->cblk_w_log2 = r->cblk_h_log2 = 6;
    r->nprecincts = 3;
    r->prec_w_log2[0] = r->prec_h_log2[0] = 8;
    r->prec_w_log2[1] = r->prec_h_log2[1] = 8;
    r->prec_w_log2[2] = r->prec_h_log2[2] = 7;
    r->progression = 2;
    r->sop = r->eph = r->plt = r->tparts_r = 1;
    r->guard_bits = 1;
    bool lossless = conversion == JP2HIP_LOSSLESS;
    r->reversible = lossless ? 1 : 0;
    r->mct = 1;
    r->qstep = 1.0 / 256.0;
    r->rate_bpp = lossless ? 0.0 : 3.0;
    r->format = JP2HIP_FORMAT_JPX;
    r->comment = 1;
    r->slope_skip = 1;
    r->flush_period = 1024;
}

// Slope prediction's rate target (bytes; 0 = prediction off) -- the same
// floor(rate * W * H / 8) the oracle's predict_and_code uses.
int64_t skip_target_of(const jp2hip_recipe &rc, int w, int h) {
    if (!rc.slope_skip || rc.rate_bpp <= 0.0) return 0;
    return (int64_t)std::floor(rc.rate_bpp * (double)w * (double)h / 8.0);
}

// A caller-supplied layout (jp2hip_encode_device*) is checked against the
// source buffer before any kernel reads it: the strips that rows [row0, row1)
// touch must lie inside src_len (uncompressed), tiles must hold a whole tile
// (uncompressed tiled), and compressed strips are checked in
// unpack_if_compressed.
bool validate_layout(const jp2hip_layout *lay, size_t src_len, int row0, int row1, std::string &err) {
    if (lay->width <= 0 || lay->height <= 0 || lay->components < 1 || lay->components > 4 ||
        (lay->bits != 8 && lay->bits != 16) || (lay->planar != 1 && lay->planar != 2) || lay->rows_per_strip <= 0 ||
        lay->nstrips <= 0 || !lay->strip_offsets) {
        err = "layout: bad geometry or strip table";
        return false;
    }
    const uint64_t spp_row = lay->planar == 2 ? 1 : (uint64_t)lay->components;
    const uint64_t px = spp_row * (uint64_t)(lay->bits / 8);
    const int planes = lay->planar == 2 ? lay->components : 1;
    if (lay->tile_width > 0 || lay->tile_height > 0) {
        if (lay->tile_width <= 0 || lay->tile_height <= 0 || !lay->strip_bytes) {
            err = "layout: tiles need tile_width, tile_height and strip_bytes";
            return false;
        }
        const int64_t across = (lay->width + lay->tile_width - 1) / lay->tile_width;
        const int64_t need = across * ((lay->height + lay->tile_height - 1) / lay->tile_height) * planes;
        if (need > lay->nstrips) { err = "layout: too few tiles"; return false; }
        const uint64_t unit = (uint64_t)lay->tile_width * lay->tile_height * px;
        for (int64_t i = 0; i < need; i++) {
            const uint64_t o = lay->strip_offsets[i], n = lay->strip_bytes[i];
            if (o > src_len || n > src_len - o || (lay->compression <= 1 && n < unit)) {
                err = "layout: tile " + std::to_string(i) + " lies outside the source buffer or is short";
                return false;
            }
        }
        return true;
    }
    if (lay->compression > 1) return true;  // checked with the strip byte counts in unpack_if_compressed
    const int64_t per_plane = (lay->height + (int64_t)lay->rows_per_strip - 1) / lay->rows_per_strip;
    if (per_plane * planes > lay->nstrips) { err = "layout: too few strips"; return false; }
    const uint64_t row_bytes = (uint64_t)lay->width * px;
    const int64_t s0 = std::max(0, row0) / lay->rows_per_strip;
    const int64_t s1 = std::min<int64_t>(per_plane, ((int64_t)std::min(row1, lay->height) + lay->rows_per_strip - 1) /
                                                        lay->rows_per_strip);
    for (int p = 0; p < planes; p++)
        for (int64_t s = s0; s < s1; s++) {
            const uint64_t o = lay->strip_offsets[(size_t)(p * per_plane + s)];
            const uint64_t rows = (uint64_t)std::min<int64_t>(lay->rows_per_strip, lay->height - s * lay->rows_per_strip);
            if (o > src_len || rows * row_bytes > src_len - o) {
                err = "layout: strip " + std::to_string(p * per_plane + s) + " lies outside the source buffer";
                return false;
            }
        }
    return true;
}

// LZW / Deflate / PackBits strips are decoded on the GPU into the context's staging
// buffer first; afterwards (d_src, lay) describe uncompressed strips.
bool unpack_if_compressed(jp2hip_ctx *ctx, const void *&d_src, size_t src_len, const jp2hip_layout *&lay,
                          jp2hip_layout &ulay, std::vector<uint64_t> &uoffs, std::string &err) {
    if (lay->compression <= 1 && lay->tile_width <= 0) return true;
    if (lay->compression > 1 && lay->compression != 5 && lay->compression != 8 && lay->compression != 32946 &&
        lay->compression != 32773) {
        err = "layout: compression " + std::to_string(lay->compression) + " is not supported";
        return false;
    }
    if (!lay->strip_bytes || !lay->strip_offsets || lay->nstrips <= 0 || lay->rows_per_strip <= 0 ||
        (lay->tile_width > 0) != (lay->tile_height > 0)) {
        err = "layout: compressed strips / tiles need strip_offsets and strip_bytes";
        return false;
    }
    for (int i = 0; i < lay->nstrips; i++)  // the decoders trust these bounds
        if (lay->strip_offsets[i] > src_len || lay->strip_bytes[i] > src_len - lay->strip_offsets[i]) {
            err = "layout: compressed strip " + std::to_string(i) + " lies outside the source buffer";
            return false;
        }
    const void *d2 = nullptr;
    if (!ctx->gpu.unpack_strips(d_src, *lay, ulay, uoffs, &d2, err)) return false;
    d_src = d2;
    lay = &ulay;
    return true;
}

// Tile-split with compressed or tiled strips (a rank's band of a BigTIFF
// master): only the strips / tiles that image rows [row0, row1) touch are
// decoded -- as a stand-alone image of their rows [R0, R1) -- and the result
// is described as a full-image layout of uncompressed strips whose entries
// outside the band are never read (the sub-plan reads only its rows).  Only
// the band's units must lie inside d_src, as for uncompressed strips.
bool unpack_band(jp2hip_ctx *ctx, const void *&d_src, size_t src_len, const jp2hip_layout *&lay, int row0, int row1,
                 jp2hip_layout &ulay, std::vector<uint64_t> &uoffs, std::string &err) {
    if (lay->compression <= 1 && lay->tile_width <= 0) return true;
    const bool tiled = lay->tile_width > 0;
    if (lay->width <= 0 || lay->height <= 0 || !lay->strip_offsets || !lay->strip_bytes ||
        (tiled && lay->tile_height <= 0) || (!tiled && lay->rows_per_strip <= 0) || (lay->planar != 1 && lay->planar != 2) ||
        lay->components < 1 || (lay->bits != 8 && lay->bits != 16)) {
        err = "layout: compressed strips / tiles need a geometry, strip_offsets and strip_bytes";
        return false;
    }
    const int uh = tiled ? lay->tile_height : lay->rows_per_strip;  // rows per unit
    const int planes = lay->planar == 2 ? lay->components : 1;
    const int64_t across = tiled ? (lay->width + lay->tile_width - 1) / lay->tile_width : 1;
    const int64_t urows = (lay->height + (int64_t)uh - 1) / uh;  // unit rows per plane
    const int64_t per_plane = across * urows;
    if (per_plane * planes > lay->nstrips) {
        err = tiled ? "layout: too few tiles" : "layout: too few strips";
        return false;
    }
    const int64_t u0 = std::max(0, row0) / uh;
    const int64_t u1 = std::min<int64_t>(urows, ((int64_t)std::min(row1, lay->height) + uh - 1) / uh);
    if (u1 <= u0) {
        err = "layout: empty band";
        return false;
    }
    const int R0 = (int)(u0 * uh), R1 = (int)std::min<int64_t>(lay->height, u1 * uh);
    const uint64_t px = (uint64_t)(lay->planar == 2 ? 1 : lay->components) * (uint64_t)(lay->bits / 8);
    const uint64_t unit = tiled ? (uint64_t)lay->tile_width * lay->tile_height * px : 0;
    std::vector<uint64_t> voff, vcnt;
    for (int p = 0; p < planes; p++)
        for (int64_t u = u0; u < u1; u++)
            for (int64_t x = 0; x < across; x++) {
                const size_t i = (size_t)(p * per_plane + u * across + x);
                const uint64_t o = lay->strip_offsets[i], n = lay->strip_bytes[i];
                if (o > src_len || n > src_len - o || (lay->compression <= 1 && n < unit)) {
                    err = "layout: strip / tile " + std::to_string(i) + " of the band lies outside the source buffer";
                    return false;
                }
                voff.push_back(o);
                vcnt.push_back(n);
            }
    jp2hip_layout v = *lay;
    v.height = R1 - R0;
    v.nstrips = (int32_t)voff.size();
    v.strip_offsets = voff.data();
    v.strip_bytes = vcnt.data();
    jp2hip_layout vu;
    std::vector<uint64_t> vuoffs;
    const void *d2 = nullptr;
    if (!ctx->gpu.unpack_strips(d_src, v, vu, vuoffs, &d2, err)) return false;
    // the full-image view: unit row u of plane p at its decoded place
    const uint64_t row_bytes = (uint64_t)lay->width * px;
    ulay = vu;
    ulay.height = lay->height;
    ulay.rows_per_strip = uh;
    ulay.nstrips = (int32_t)(urows * planes);
    uoffs.assign((size_t)(urows * planes), 0);
    for (int p = 0; p < planes; p++)
        for (int64_t u = u0; u < u1; u++)
            uoffs[(size_t)(p * urows + u)] = tiled ? vuoffs[(size_t)p] + (uint64_t)(u - u0) * uh * row_bytes
                                                   : vuoffs[(size_t)(p * (u1 - u0) + (u - u0))];
    ulay.strip_offsets = uoffs.data();
    d_src = d2;
    lay = &ulay;
    return true;
}

// Kdu-Layer-Info byte counts: the code-stream through each layer.
void layer_end_of(const jp2hip::Plan &P, int64_t tp_hdr_bytes, const int64_t *layer_bytes, int64_t *layer_end) {
    std::vector<uint8_t> mh;
    jp2hip::main_header(P, mh, nullptr, nullptr);
    int64_t acc = (int64_t)mh.size() + tp_hdr_bytes;
    for (int l = 0; l < P.rc.layers; l++) {
        acc += layer_bytes[l];
        layer_end[l] = acc;
    }
}

void fill_stats(jp2hip_stats *stats, const jp2hip::StageTimes &st, double t_start, double h2d_ms, int64_t nb,
                const jp2hip::T2Summary &sum, int64_t out_bytes, int iters, int waits) {
    if (!stats) return;
    std::memset(stats, 0, sizeof *stats);
    stats->total_ms = now_ms() - t_start;
    stats->h2d_ms = h2d_ms;
    stats->ingest_ms = st.ingest;
    stats->dwt_ms = st.dwt;
    stats->quant_ms = st.quant;
    stats->t1_ms = st.t1_cm + st.t1_mq;
    stats->t1_cm_ms = st.t1_cm;
    stats->t1_mq_ms = st.t1_mq;
    stats->pcrd_ms = st.pcrd;
    stats->d2h_ms = st.d2h;
    stats->t2_ms = st.t2;
    stats->codeblocks = nb;
    stats->t1_bytes = sum.t1_bytes;
    stats->coded_passes = sum.coded_passes;
    stats->out_bytes = out_bytes;
    stats->rate_iterations = iters;
    stats->host_waits = waits;
    stats->mq_decisions = sum.decisions;
    stats->stream_need_bytes = sum.stream_need;
}

// The caller's recipe (or the default for `conversion`) with its padding
// bytes zeroed, so PlanCache's byte compare sees only the fields.
jp2hip_recipe recipe_of(const jp2hip_recipe *recipe, int conversion) {
    jp2hip_recipe rc;
    std::memset(&rc, 0, sizeof rc);
    if (recipe) rc = *recipe;
    else default_recipe(&rc, conversion);
    const size_t gap0 = offsetof(jp2hip_recipe, mct) + sizeof rc.mct, gap1 = offsetof(jp2hip_recipe, qstep);
    if (gap1 > gap0) std::memset((char *)&rc + gap0, 0, gap1 - gap0);
    static_assert(offsetof(jp2hip_recipe, flush_period) + sizeof(int32_t) == sizeof(jp2hip_recipe),
                  "jp2hip_recipe: no tail padding");
    return rc;
}

// The whole encode with the source already in device memory.  On success
// *out is the complete file in a pinned buffer from this library's pool
// (out_alloc; released with jp2hip_free).  Everything up to the
// code-stream bytes runs on the GPU (tier-2 included, t2_device.hip); the host picks
// the rate-control budgets from one small summary per pass and writes the
// file and main headers.
int encode_core(jp2hip_ctx *ctx, const void *d_src, size_t src_len, const jp2hip_layout *lay,
                int conversion, const jp2hip_recipe *recipe, uint8_t **out, size_t *out_len,
                jp2hip_stats *stats, double t_start, double h2d_ms) {
    using namespace jp2hip;
    if (conversion != JP2HIP_LOSSY && conversion != JP2HIP_LOSSLESS)
        return fail("conversion must be JP2HIP_LOSSY (0) or JP2HIP_LOSSLESS (1)");
    const jp2hip_recipe rc = recipe_of(recipe, conversion);
    if (!lay || !d_src) return fail("null source or layout");
    ctx->gpu.take_waits();  // count this encode's host waits (stats)
    ctx->gpu.begin_encode();
    EncodeEnd end{ctx};
    std::string err;
    jp2hip_layout ulay;
    std::vector<uint64_t> uoffs;
    if (!validate_layout(lay, src_len, 0, lay->height, err)) return fail(err);
    if (!unpack_if_compressed(ctx, d_src, src_len, lay, ulay, uoffs, err)) return fail(err);
    PlanCache &pc = ctx->pc;
    if (!pc.valid || pc.w != lay->width || pc.h != lay->height || pc.nc != lay->components || pc.bits != lay->bits ||
        std::memcmp(&pc.rc, &rc, sizeof rc) != 0) {
        pc.valid = false;
        if (!build_plan(pc.plan, rc, lay->width, lay->height, lay->components, lay->bits, err)) return fail(err);
        t2_tables(pc.plan, 0, pc.plan.ntx * pc.plan.nty, 0, pc.tabs);
        main_header(pc.plan, pc.mh0, nullptr, nullptr);
        pc.rc = rc;
        pc.w = lay->width; pc.h = lay->height; pc.nc = lay->components; pc.bits = lay->bits;
        pc.valid = true;
    }
    const Plan &plan = pc.plan;
    const bool prof = ctx->cfg.profile != 0;
    StageTimes st;
    int64_t skip_target = skip_target_of(rc, plan.w, plan.h);
    // tier-2 tables first: every host->device copy of the encode is issued
    // while the stream is idle (a copy queued behind kernels holds up the
    // copy engine for the other contexts)
    if (!ctx->gpu.t2_load(plan, pc.tabs, err)) return fail(err);
    if (!ctx->gpu.run_front(d_src, *lay, plan, prof, st, err, skip_target)) return fail(err);
    const int L = rc.layers;
    std::vector<uint8_t> mh = pc.mh0;
    T2Summary sum;
    std::memset(&sum, 0, sizeof sum);
    int iters = 0;
    int64_t cs_bytes = 0;
    if (rc.rate_bpp <= 0.0) {
        // lossless: per -flush_period stripe, layer l keeps the passes whose
        // slopes clear lossless_layer_frac(l) of the stripe's tier-1 bytes
        for (int grow = 0;; grow++) {
            if (!ctx->gpu.select_lossless(plan, err) || !ctx->gpu.t2_size(plan, true, prof, st, sum, err))
                return fail(err);
            if ((sum.err & kErrSlotPool) && grow < 2) {
                // the decision-stream pool was short: again with the size
                // this encode needed (GpuEncoder::run_front)
                if (!ctx->gpu.pool_grow(err) || !ctx->gpu.run_front(d_src, *lay, plan, prof, st, err, skip_target))
                    return fail(err);
                continue;
            }
            break;
        }
        if (sum.err) return fail("tier-1 output capacity exceeded");
        iters = 1;
        cs_bytes = (int64_t)mh.size() + sum.part_bytes + 2;
    } else {
        // the rate loop runs on the device (GpuEncoder::rate_loop): one
        // iteration per host wait, what the usual encode needs -- the first
        // budget's header estimate (16 bytes per packet) lands it under the
        // target (C2: 8 985 521 of 9 000 000 bytes); an encode whose headers
        // are heavier takes a second wait for its next iterations
        RateState init;
        std::memset(&init, 0, sizeof init);
        init.target = (int64_t)std::floor(rc.rate_bpp * (double)plan.w * (double)plan.h / 8.0);
        init.budget = init.target - 16 * plan.npackets - 16 * plan.ntileparts - 256;
        init.fixed = (int64_t)mh.size() + 2;
        init.skip_target = skip_target;
        RateState rs;
        bool restart = true;
        for (int grow = 0;;) {
            if (!ctx->gpu.rate_loop(plan, init, restart, restart ? 1 : 2, prof, st, rs, sum, err)) return fail(err);
            restart = false;
            if ((sum.err & kErrSlotPool) && grow++ < 2) {
                // the decision-stream pool was short: again with the size
                // this encode needed (GpuEncoder::run_front)
                if (!ctx->gpu.pool_grow(err) ||
                    !ctx->gpu.run_front(d_src, *lay, plan, prof, st, err, init.skip_target))
                    return fail(err);
                restart = true;
                continue;
            }
            if (sum.err) return fail("tier-1 output capacity exceeded");
            if (rs.safety) {
                // slope prediction's safety net (oracle predict_and_code):
                // planes were skipped, yet every coded byte fits -> code all
                init.skip_target = 0;
                if (!ctx->gpu.run_front(d_src, *lay, plan, prof, st, err, 0)) return fail(err);
                restart = true;
                continue;
            }
            if (rs.halt) break;
        }
        iters = rs.iters;
        cs_bytes = rs.cs_bytes;
    }
    // Kdu-Layer-Info: the final selection's slope keys (lossless: the last
    // layer takes every pass) and the code-stream bytes through each layer
    std::vector<uint64_t> K(sum.kc, sum.kc + L);
    if (rc.rate_bpp <= 0.0) K[L - 1] = 0;
    std::vector<int64_t> layer_end((size_t)L);
    layer_end_of(plan, sum.tp_hdr_bytes, sum.layer_bytes, layer_end.data());
    main_header(plan, mh, K.data(), layer_end.data());
    const size_t fh = file_header_bytes(plan);
    const size_t n = fh + (size_t)cs_bytes;
    uint8_t *buf = out_alloc(n);
    if (!buf) return fail("out of (pinned) host memory");
    write_file_header(plan, (uint64_t)cs_bytes, buf);
    std::memcpy(buf + fh, mh.data(), mh.size());
    if (!ctx->gpu.t2_emit(plan, 0, (uint64_t)sum.part_bytes, buf + fh + mh.size(), prof, st, err) ||
        !ctx->gpu.collect_profile(st, err)) {
        out_free(buf);
        return fail(err);
    }
    buf[n - 2] = 0xFF;
    buf[n - 1] = 0xD9;
    *out = buf;
    *out_len = n;
    fill_stats(stats, st, t_start, h2d_ms, (int64_t)plan.blocks.size(), sum, (int64_t)n, iters,
               ctx->gpu.take_waits());
    if (stats) {
        stats->stream_pool_bytes = (int64_t)ctx->gpu.stream_pool_bytes();
        stats->pool_grows = ctx->gpu.take_pool_grows();
    }
    end.ok = true;
    return 0;
}

// Tile-split encode (jp2hip.h, jp2hip_encode_device_split; split.cpp has the
// exchange rule).  Rank `rank` runs the device pipeline -- tier-2 included --
// on its band of tile rows only; budgets, thresholds and tier-2 sizes are
// agreed through sp->allreduce_sum so the parts concatenate to the
// single-GPU file.
int encode_split_core(jp2hip_ctx *ctx, const void *d_src, size_t src_len, const jp2hip_layout *lay, int conversion,
                      const jp2hip_recipe *recipe, const jp2hip_split *sp, uint8_t **out, size_t *out_len,
                      uint64_t *file_offset, uint64_t *file_len, jp2hip_stats *stats, double t_start) {
    using namespace jp2hip;
    if (conversion != JP2HIP_LOSSY && conversion != JP2HIP_LOSSLESS)
        return fail("conversion must be JP2HIP_LOSSY (0) or JP2HIP_LOSSLESS (1)");
    const int world = sp ? sp->world : 1, rank = sp ? sp->rank : 0;
    if (world < 1 || rank < 0 || rank >= world) return fail("split: bad rank / world");
    if (world > 1 && !sp->allreduce_sum) return fail("split: world > 1 needs an allreduce_sum callback");
    auto allreduce = [&](int64_t *v, int n) {
        return world <= 1 || sp->allreduce_sum(sp->user, v, (int32_t)n) == 0;
    };
    const jp2hip_recipe rc = recipe_of(recipe, conversion);
    if (!lay || !d_src) return fail("null source or layout");
    ctx->gpu.take_waits();
    ctx->gpu.begin_encode();
    EncodeEnd end{ctx};
    Plan full;
    std::string err;
    if (!build_plan(full, rc, lay->width, lay->height, lay->components, lay->bits, err)) return fail(err);
    int tr0, tr1;
    split_tile_rows(full.nty, rc.tile_h, full.h, rc.flush_period, rank, world, tr0, tr1);
    Plan sub;
    make_subplan(full, tr0, tr1, sub);
    const bool have = sub.ntc > 0;
    // only this rank's rows are read, so only their strips (or tiles) must be
    // in d_src; compressed / tiled units of the band are decoded here (a rank
    // that fails here still joins every exchange below)
    jp2hip_layout ulay;
    std::vector<uint64_t> uoffs;
    const bool packed = lay->compression > 1 || lay->tile_width > 0;
    bool ok = !have || (packed ? unpack_band(ctx, d_src, src_len, lay, sub.row0, sub.row0 + sub.band_h, ulay, uoffs, err)
                               : validate_layout(lay, src_len, sub.row0, sub.row0 + sub.band_h, err));
    const bool prof = ctx->cfg.profile != 0;
    StageTimes st;
    std::vector<uint64_t> keys;
    std::vector<int64_t> cum;
    // slope prediction over the whole image: the plane histogram is summed
    // over ranks (one all-reduce of kSlopeBins + 1 int64, the last a failure
    // flag, so a rank that failed earlier still joins the exchange)
    int64_t skip_target = skip_target_of(rc, full.w, full.h);
    bool hist_done = false;
    GpuEncoder::HistReduce reduce = [&](std::vector<int64_t> &h) {
        hist_done = true;
        std::vector<int64_t> v(h.size() + 1, 0);
        std::copy(h.begin(), h.end(), v.begin());
        if (!allreduce(v.data(), (int)v.size()) || v.back() != 0) return false;
        std::copy(v.begin(), v.end() - 1, h.begin());
        return true;
    };
    T2Tables tabs;  // loaded before the front (host->device copies on an idle stream)
    const int tile0 = sub.tile0, tile1 = sub.tile0 + full.ntx * (tr1 - tr0);
    if (ok && have) {
        t2_tables(full, tile0, tile1, sub.block0, tabs);
        ok = ctx->gpu.t2_load(sub, tabs, err);
    }
    ok = ok && (!have || ctx->gpu.run_front(d_src, *lay, sub, prof, st, err, skip_target, &reduce, true));
    if (skip_target > 0 && !hist_done) {  // no blocks here, or failed before the exchange
        std::vector<int64_t> v((size_t)kSlopeBins + 1, 0);
        v.back() = ok ? 0 : 1;
        if (!allreduce(v.data(), (int)v.size())) return fail("split: all-reduce failed");
        if (ok && v.back()) { ok = false; err = "split: another rank failed"; }
    }
    const int L = rc.layers;
    std::vector<int64_t> budgets((size_t)L, 0);
    std::vector<uint64_t> K((size_t)L);
    int iters = 0;
    int64_t cs_bytes = 0;
    T2Summary sum;
    std::memset(&sum, 0, sizeof sum);
    int64_t g_tp_hdr = 0;                          // whole-image sums of the last pass
    std::vector<int64_t> g_layer((size_t)L, 0);    // (Kdu-Layer-Info)
    std::vector<uint8_t> mh;
    main_header(full, mh, nullptr, nullptr);
    // one selection + tier-2 sizing pass for `budgets`; false on failure
    auto round = [&]() -> bool {
        if (jp2hip_split_thresholds(keys.data(), cum.data(), (int64_t)keys.size(), budgets.data(), L, sp,
                                    K.data()) != 0) {
            err = "split: threshold exchange failed";
            return false;
        }
        bool rok = true;
        if (have) rok = ctx->gpu.select_keys(sub, K, err) && ctx->gpu.t2_size(sub, false, prof, st, sum, err);
        if (rok && have && sum.err) { rok = false; err = "tier-1 output capacity exceeded"; }
        // [0] part bytes, [1] failure flag, [2] tile-part header bytes,
        // [3..] packet bytes per layer (Kdu-Layer-Info)
        std::vector<int64_t> v((size_t)L + 3, 0);
        v[1] = rok ? 0 : 1;
        if (rok && have) {
            v[0] = sum.part_bytes;
            v[2] = sum.tp_hdr_bytes;
            for (int l = 0; l < L; l++) v[3 + l] = sum.layer_bytes[l];
        }
        if (!allreduce(v.data(), (int)v.size())) { err = "split: all-reduce failed"; return false; }
        if (v[1]) { if (rok) err = "split: another rank failed"; return false; }
        cs_bytes = (int64_t)mh.size() + 2 + v[0];
        g_tp_hdr = v[2];
        g_layer.assign(v.begin() + 3, v.end());
        iters++;
        return true;
    };
    for (int attempt = 0; attempt < 2; attempt++) {
        if (attempt == 1) {  // the prediction's safety net, decided globally (below)
            keys.clear();
            cum.clear();
            ok = !have || ctx->gpu.run_front(d_src, *lay, sub, prof, st, err, 0, nullptr, true);
            skip_target = 0;
            iters = 0;
        }
        if (rc.rate_bpp <= 0.0) {
            // lossless: every -flush_period stripe's layers come from its own
            // tier-1 bytes (the plan's rate-control groups; a rank holds
            // whole stripes), so the selection needs no exchange -- only the
            // part sizes, the Kdu-Layer-Info bytes and each layer's slope
            // key (the largest over the ranks' stripes) are shared
            bool rok = ok && (!have || (ctx->gpu.select_lossless(sub, err) && ctx->gpu.t2_size(sub, true, prof, st, sum, err)));
            if (rok && have && sum.err) {
                rok = false;
                err = "tier-1 output capacity exceeded";
            }
            std::vector<int64_t> v((size_t)L + 3 + (size_t)world * L, 0);
            v[1] = rok ? 0 : 1;
            if (rok && have) {
                v[0] = sum.part_bytes;
                v[2] = sum.tp_hdr_bytes;
                for (int l = 0; l < L; l++) {
                    v[3 + l] = sum.layer_bytes[l];
                    v[3 + L + (size_t)rank * L + l] = (int64_t)sum.kc[l];  // (keys of positive doubles: < 2^63)
                }
            }
            if (!allreduce(v.data(), (int)v.size())) return fail("split: all-reduce failed");
            if (v[1]) return fail(rok ? std::string("split: another rank failed") : err);
            cs_bytes = (int64_t)mh.size() + 2 + v[0];
            g_tp_hdr = v[2];
            g_layer.assign(v.begin() + 3, v.begin() + 3 + L);
            for (int l = 0; l < L; l++) {
                K[l] = 0;
                for (int r = 0; r < world; r++) K[l] = std::max(K[l], (uint64_t)v[3 + L + (size_t)r * L + l]);
            }
            iters = 1;
            break;
        }
        ok = ok && (!have || ctx->gpu.segments(sub, keys, cum, err));
        {
            int64_t flag = ok ? 0 : 1;
            if (!allreduce(&flag, 1)) return fail("split: all-reduce failed");
            if (!ok) return fail(err);
            if (flag) return fail("split: another rank failed");
        }
        const int64_t target = (int64_t)std::floor(rc.rate_bpp * (double)full.w * (double)full.h / 8.0);
        int64_t budget = target - 16 * full.npackets - 16 * full.ntileparts - 256;
        bool rerun = false;
        for (int it = 0; it < 8; it++) {
            if (budget < 0) budget = 0;
            for (int l = 0; l < L; l++) budgets[l] = budget >> (L - 1 - l);
            if (!round()) return fail(err);
            if (it == 0 && skip_target > 0) {
                int64_t v[2] = {have ? sum.t1_bytes : 0, have ? sum.skipped : 0};
                if (!allreduce(v, 2)) return fail("split: all-reduce failed");
                if (v[1] && v[0] < skip_target) { rerun = true; break; }
            }
            if (cs_bytes <= target) break;
            budget -= ((cs_bytes - target) << it) + ((cs_bytes - target) >> 4) + 64;  // as encode_core
        }
        if (!rerun) break;
    }
    // this rank's part of the file
    const bool with_main = rank == 0, with_eoc = rank == world - 1;
    const size_t fh = with_main ? file_header_bytes(full) : 0;
    const uint64_t head = with_main ? fh + mh.size() : 0;
    const uint64_t part = head + (uint64_t)(have ? sum.part_bytes : 0) + (with_eoc ? 2 : 0);
    // everything this rank's emission allocates is allocated before the
    // ranks agree on the part sizes, so a rank that cannot fails with the
    // others (the failure slot sizes[world]); a HIP error in the emission
    // itself, after the exchange, fails this rank alone: the caller treats
    // any rank's failure as the encode's (jp2hip.h)
    uint8_t *buf = out_alloc(part ? part : 1);
    bool ready = buf != nullptr;
    if (!ready) err = "out of (pinned) host memory";
    if (ready && have) ready = ctx->gpu.t2_reserve(sum.part_bytes, err);
    std::vector<int64_t> sizes((size_t)world + 1, 0);
    sizes[rank] = (int64_t)part;
    sizes[world] = ready ? 0 : 1;
    if (!allreduce(sizes.data(), world + 1)) {
        out_free(buf);
        return fail("split: all-reduce failed");
    }
    if (sizes[world]) {
        out_free(buf);
        return fail(ready ? std::string("split: another rank failed") : err);
    }
    uint64_t off = 0, flen = 0;
    for (int r = 0; r < world; r++) {
        if (r < rank) off += (uint64_t)sizes[r];
        flen += (uint64_t)sizes[r];
    }
    if (with_main) {
        std::vector<uint64_t> Kcom = K;
        if (rc.rate_bpp <= 0.0) Kcom[L - 1] = 0;
        std::vector<int64_t> layer_end((size_t)L);
        layer_end_of(full, g_tp_hdr, g_layer.data(), layer_end.data());
        main_header(full, mh, Kcom.data(), layer_end.data());
        write_file_header(full, (uint64_t)cs_bytes, buf);
        std::memcpy(buf + fh, mh.data(), mh.size());
    }
    if (have && (!ctx->gpu.t2_emit(sub, 0, (uint64_t)sum.part_bytes, buf + head, prof, st, err) ||
                 !ctx->gpu.collect_profile(st, err))) {
        out_free(buf);
        return fail(err);
    }
    if (with_eoc) {
        buf[part - 2] = 0xFF;
        buf[part - 1] = 0xD9;
    }
    *out = buf;
    *out_len = part;
    if (file_offset) *file_offset = off;
    if (file_len) *file_len = flen;
    fill_stats(stats, st, t_start, 0.0, (int64_t)sub.blocks.size(), sum, (int64_t)flen, iters,
               ctx->gpu.take_waits());
    if (stats) {
        stats->stream_pool_bytes = (int64_t)ctx->gpu.stream_pool_bytes();
        stats->pool_grows = ctx->gpu.take_pool_grows();
    }
    end.ok = true;
    return 0;
}

// ---- tile-split inside the library (jp2hip_split_peers) ----
// The ranks of one encode are threads of this process, one per member
// context (each with its own GPU and stream); their exchanges (split.cpp,
// encode_split_core) are summed here on the host: a few hundred vectors of at
// most 1 025 int64 per image, nothing that needs RCCL.  A rank that fails
// before an exchange, or returns, aborts the group, so no rank waits forever
// in an exchange another rank will never join.
class HostGroup {
  public:
    explicit HostGroup(int world) : world_(world) {}
    int reduce(int64_t *v, int n) {
        std::unique_lock<std::mutex> lk(mu_);
        if (aborted_) return -1;
        if (n < 0) {  // a bug in the caller: fail every rank, not just this one
            aborted_ = true;
            cv_.notify_all();
            return -1;
        }
        if (arrived_ == 0) {
            acc_.assign((size_t)n, 0);
            n_ = n;
        } else if (n != n_) {  // ranks out of step: a bug, never a wrong sum
            aborted_ = true;
            cv_.notify_all();
            return -1;
        }
        for (int i = 0; i < n; i++) acc_[(size_t)i] += v[i];
        const uint64_t g = gen_;
        if (++arrived_ == world_) {
            res_[g & 1].swap(acc_);  // generation g+2 reuses it only after every rank copied it
            arrived_ = 0;
            gen_++;
            cv_.notify_all();
        } else {
            cv_.wait(lk, [&] { return gen_ != g || aborted_; });
            if (gen_ == g) return -1;  // aborted before this exchange completed
        }
        std::copy(res_[g & 1].begin(), res_[g & 1].begin() + n, v);
        return 0;
    }
    void abort() {
        std::lock_guard<std::mutex> lk(mu_);
        aborted_ = true;
        cv_.notify_all();
    }
    static int call(void *user, int64_t *v, int32_t n) { return static_cast<HostGroup *>(user)->reduce(v, n); }

  private:
    std::mutex mu_;
    std::condition_variable cv_;
    int world_, arrived_ = 0, n_ = 0;
    uint64_t gen_ = 0;
    bool aborted_ = false;
    std::vector<int64_t> acc_, res_[2];
};

// The strips (or compressed strips / tiles, whole) that image rows
// [row0, row1) read, as (file offset, bytes, strip-table index): what one rank
// uploads.  The C++ form of jp2hip.split.band_strips.
struct BandCopy {
    uint64_t src, n;
    size_t idx;
};
bool band_units(const jp2hip_layout &lay, size_t flen, int row0, int row1, std::vector<BandCopy> &cp,
                std::string &err) {
    cp.clear();
    if (row1 <= row0) return true;
    const bool packed = lay.compression > 1 || lay.tile_width > 0, tiled = lay.tile_width > 0;
    const int uh = tiled ? lay.tile_height : lay.rows_per_strip;
    if (uh <= 0 || lay.width <= 0 || lay.height <= 0 || (packed && !lay.strip_bytes) || !lay.strip_offsets) {
        err = "layout: bad strip table";
        return false;
    }
    const int planes = lay.planar == 2 ? lay.components : 1;
    const int64_t across = tiled ? (lay.width + (int64_t)lay.tile_width - 1) / lay.tile_width : 1;
    const int64_t urows = (lay.height + (int64_t)uh - 1) / uh, per_plane = across * urows;
    if (per_plane * planes > lay.nstrips) {
        err = tiled ? "layout: too few tiles" : "layout: too few strips";
        return false;
    }
    const uint64_t row_bytes = (uint64_t)lay.width * (uint64_t)(lay.planar == 2 ? 1 : lay.components) * (lay.bits / 8);
    const int64_t u0 = row0 / uh, u1 = std::min<int64_t>(urows, (row1 + (int64_t)uh - 1) / uh);
    for (int p = 0; p < planes; p++)
        for (int64_t u = u0; u < u1; u++)
            for (int64_t x = 0; x < across; x++) {
                const size_t i = (size_t)(p * per_plane + u * across + x);
                const uint64_t o = lay.strip_offsets[i];
                const uint64_t n = packed ? lay.strip_bytes[i]
                                          : (uint64_t)std::min<int64_t>(uh, lay.height - u * uh) * row_bytes;
                if (o > flen || n > flen - o) {
                    err = "tiff: strip " + std::to_string(i) + " out of range";
                    return false;
                }
                cp.push_back({o, n, i});
            }
    return true;
}

struct RankResult {
    int rc = -1;
    std::string err;
    uint8_t *part = nullptr;
    size_t part_len = 0;
    uint64_t off = 0, flen = 0;
    jp2hip_stats st;
};

// One rank of a host-driven tile-split: gather the band's strips from the
// TIFF in host memory into pinned memory, upload them to member `m`, run the
// split encode, and (fd >= 0) write the part at its offset of the output file.
void split_rank(jp2hip_ctx *m, int rank, int world, HostGroup &grp, const uint8_t *file, size_t flen,
                const jp2hip_layout &lay, int conversion, const jp2hip_recipe &rc, int fd, double t0,
                RankResult &o) {
    std::memset(&o.st, 0, sizeof o.st);
    int r0 = 0, r1 = 0;
    jp2hip_split_rows(lay.height, rc.tile_h, rc.flush_period, rank, world, &r0, &r1);
    std::vector<BandCopy> cp;
    if (!band_units(lay, flen, r0, r1, cp, o.err)) {
        grp.abort();
        return;
    }
    size_t tot = 0;
    for (const BandCopy &c : cp) tot += c.n;
    uint8_t *h = out_alloc(std::max<size_t>(tot, 1));  // pinned: the upload is one DMA
    if (!h) {
        o.err = "out of (pinned) host memory";
        grp.abort();
        return;
    }
    const bool packed = lay.compression > 1 || lay.tile_width > 0;
    std::vector<uint64_t> offs((size_t)lay.nstrips * (packed ? 2 : 1), 0);
    size_t pos = 0;
    for (const BandCopy &c : cp) {
        std::memcpy(h + pos, file + c.src, c.n);
        offs[c.idx] = pos;
        if (packed) offs[(size_t)lay.nstrips + c.idx] = c.n;
        pos += c.n;
    }
    jp2hip_layout bl = lay;
    bl.strip_offsets = offs.data();
    bl.strip_bytes = packed ? offs.data() + lay.nstrips : nullptr;
    {
        std::lock_guard<std::mutex> lk(m->mu);
        if (!m->gpu.upload_source(h, std::max<size_t>(tot, 1), o.err) || !m->gpu.check_residency(o.err)) {
            grp.abort();
        } else {
            jp2hip_split sp{rank, world, &HostGroup::call, &grp};
            o.rc = encode_split_core(m, m->gpu.source(), std::max<size_t>(tot, 1), &bl, conversion, &rc, &sp,
                                     &o.part, &o.part_len, &o.off, &o.flen, &o.st, t0);
            if (o.rc != 0) o.err = g_err;
            grp.abort();  // harmless after the last exchange; wakes the others after a failure
        }
        (void)hipStreamSynchronize(m->gpu.get_stream());  // the upload has read `h`
    }
    out_free(h);
    if (o.rc == 0 && fd >= 0) {
        size_t done = 0;
        while (done < o.part_len) {
            const ssize_t k = pwrite(fd, o.part + done, o.part_len - done, (off_t)(o.off + done));
            if (k <= 0) {
                o.rc = -1;
                o.err = "cannot write output";
                break;
            }
            done += (size_t)k;
        }
    }
}

// A whole-image encode split across ctx (rank 0) and its peers: the TIFF
// bytes are in host memory; the result goes to `fd` (each rank writes its
// part) or, fd < 0, into one pinned buffer *out.
int encode_split_host(jp2hip_ctx *ctx, const uint8_t *file, size_t flen, const jp2hip_layout &lay, int conversion,
                      const jp2hip_recipe *recipe, int fd, uint8_t **out, size_t *out_len, jp2hip_stats *stats,
                      double t0) {
    if (conversion != JP2HIP_LOSSY && conversion != JP2HIP_LOSSLESS)
        return fail("conversion must be JP2HIP_LOSSY (0) or JP2HIP_LOSSLESS (1)");
    const jp2hip_recipe rc = recipe_of(recipe, conversion);
    std::lock_guard<std::mutex> split_lk(ctx->split_mu);
    std::vector<jp2hip_ctx *> members{ctx};
    members.insert(members.end(), ctx->peers.begin(), ctx->peers.end());
    const int world = (int)members.size();
    HostGroup grp(world);
    std::vector<RankResult> res((size_t)world);
    std::vector<std::thread> th;
    for (int r = 1; r < world; r++)
        th.emplace_back([&, r] {
            split_rank(members[(size_t)r], r, world, grp, file, flen, lay, conversion, rc, fd, t0, res[(size_t)r]);
        });
    split_rank(ctx, 0, world, grp, file, flen, lay, conversion, rc, fd, t0, res[0]);
    for (std::thread &t : th) t.join();
    // report the rank that failed first-hand, not one that saw the abort
    const RankResult *bad = nullptr;
    for (const RankResult &r : res)
        if (r.rc != 0 && (!bad || (bad->err.rfind("split:", 0) == 0 && r.err.rfind("split:", 0) != 0))) bad = &r;
    if (bad) {
        const std::string e = bad->err.empty() ? "split: encode failed" : bad->err;
        for (RankResult &r : res) out_free(r.part);
        return fail(e);
    }
    const uint64_t total = res[0].flen;
    if (fd < 0) {
        uint8_t *buf = out_alloc((size_t)total);
        if (!buf) {
            for (RankResult &r : res) out_free(r.part);
            return fail("out of (pinned) host memory");
        }
        for (const RankResult &r : res) std::memcpy(buf + r.off, r.part, r.part_len);
        *out = buf;
        *out_len = (size_t)total;
    }
    for (RankResult &r : res) out_free(r.part);
    if (stats) {
        *stats = res[0].st;
        for (int r = 1; r < world; r++) {
            stats->codeblocks += res[(size_t)r].st.codeblocks;
            stats->coded_passes += res[(size_t)r].st.coded_passes;
            stats->t1_bytes += res[(size_t)r].st.t1_bytes;
            stats->mq_decisions += res[(size_t)r].st.mq_decisions;
            stats->host_waits = std::max(stats->host_waits, res[(size_t)r].st.host_waits);
        }
        stats->out_bytes = (int64_t)total;
        stats->total_ms = now_ms() - t0;
    }
    return 0;
}

bool wants_split(const jp2hip_ctx *ctx, const jp2hip_layout &lay) {
    return !ctx->peers.empty() && (int64_t)lay.width * lay.height >= ctx->split_min_pixels;
}

// A read-only mapping of a whole file (the split path reads each rank's band
// of a multi-GB TIFF straight from the page cache, in parallel).
struct MappedFile {
    int fd = -1;
    const uint8_t *p = nullptr;
    size_t n = 0;
    bool open(const char *path) {
        fd = ::open(path, O_RDONLY | O_CLOEXEC);
        if (fd < 0) return false;
        struct stat sb;
        if (fstat(fd, &sb) != 0 || sb.st_size <= 0) return false;
        n = (size_t)sb.st_size;
        void *m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
        if (m == MAP_FAILED) return false;
        p = (const uint8_t *)m;
        return true;
    }
    ~MappedFile() {
        if (p) munmap((void *)p, n);
        if (fd >= 0) ::close(fd);
    }
};

std::string temp_name(const char *out_path) {
    return std::string(out_path) + ".part-" + std::to_string((long)getpid()) + "-" +
           std::to_string((unsigned long)std::hash<std::thread::id>()(std::this_thread::get_id()) % 100000);
}

}  // namespace

extern "C" {

const char *jp2hip_version(void) { return "jp2hip 0.1.0 (gfx950)"; }

const char *jp2hip_last_error(void) { return g_err.c_str(); }

int jp2hip_probe(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return 0;
    for (int i = 0; i < n; i++) {
        hipDeviceProp_t p;
        if (hipGetDeviceProperties(&p, i) == hipSuccess && std::strncmp(p.gcnArchName, "gfx950", 6) == 0)
            return 1;
    }
    return 0;
}

int jp2hip_device_ordinals(int32_t *ordinals, int32_t max) {
    int n = 0, k = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return 0;
    for (int i = 0; i < n; i++) {
        hipDeviceProp_t p;
        if (hipGetDeviceProperties(&p, i) == hipSuccess && std::strncmp(p.gcnArchName, "gfx950", 6) == 0) {
            if (ordinals && k < max) ordinals[k] = i;
            k++;
        }
    }
    return k;
}

int jp2hip_device_count(void) { return jp2hip_device_ordinals(nullptr, 0); }

void jp2hip_recipe_init(jp2hip_recipe *recipe, int conversion) {
    if (recipe) default_recipe(recipe, conversion);
}

// Every context alive in the process, by device: an allocation that fails
// for lack of device memory takes back the buffers of idle contexts of its
// device (GpuEncoder::reclaim -> reclaim_idle).  A context is idle when its
// lock is free (no encode in it); its buffers are rebuilt by its next encode.
static std::mutex g_reg_mu;
static std::vector<jp2hip_ctx *> g_reg;

static bool reclaim_idle(jp2hip_ctx *self) {
    bool freed = false;
    std::lock_guard<std::mutex> lk(g_reg_mu);
    for (jp2hip_ctx *c : g_reg) {
        if (c == self || c->cfg.device != self->cfg.device) continue;
        std::unique_lock<std::mutex> cl(c->mu, std::try_to_lock);
        if (!cl.owns_lock() || c->gpu.device_bytes() == 0) continue;
        c->gpu.quiesce();
        freed = c->gpu.trim(0) || freed;
        c->reclaimed++;
    }
    return freed;
}

const char *jp2hip_env_check(void) {
    thread_local std::string msg;
    msg.clear();
    const char *q = std::getenv("GPU_MAX_HW_QUEUES");
    const int queues = q && *q ? std::atoi(q) : 4;  // HIP's default
    const int live = g_live_contexts.load();
    if (live > queues)
        msg += "GPU_MAX_HW_QUEUES=" + std::to_string(queues) + " is below the " + std::to_string(live) +
               " contexts of this process (contexts sharing a hardware queue run their kernels one after "
               "another; set it to contexts per GPU + 4 before the library loads); ";
    if (!msg.empty()) msg.resize(msg.size() - 2);
    return msg.c_str();
}

int jp2hip_create(jp2hip_ctx **out, const jp2hip_config *cfg) {
    if (!out) return fail("null output pointer");
    *out = nullptr;
    jp2hip_ctx *c = new (std::nothrow) jp2hip_ctx();
    if (!c) return fail("out of memory");
    std::memset(&c->cfg, 0, sizeof c->cfg);
    if (cfg) c->cfg = *cfg;
    int hw = (int)std::thread::hardware_concurrency();
    c->threads = c->cfg.host_threads > 0 ? c->cfg.host_threads : std::max(1, std::min(16, hw));
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        delete c;
        return fail("no HIP device visible (libjp2hip needs an MI355X / gfx950)");
    }
    if (c->cfg.device < 0 || c->cfg.device >= ndev) {
        delete c;
        return fail("device ordinal " + std::to_string(c->cfg.device) + " out of range (" + std::to_string(ndev) +
                    " visible)");
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, c->cfg.device) != hipSuccess ||
        std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        delete c;
        return fail("device " + std::to_string(c->cfg.device) + " is not a gfx950 (MI355X) device");
    }
    std::string err;
    if (!c->gpu.init(c->cfg.device, err)) {
        delete c;
        return fail(err);
    }
    size_t fr = 0, tot = 0;
    c->dev_total = hipMemGetInfo(&fr, &tot) == hipSuccess ? tot : 0;  // (init selected the device)
    c->gpu.reclaim = [c] { return reclaim_idle(c); };
    {
        std::lock_guard<std::mutex> lk(g_reg_mu);
        g_reg.push_back(c);
    }
    *out = c;
    g_live_contexts++;
    return 0;
}

int64_t jp2hip_device_bytes(jp2hip_ctx *ctx) {
    if (!ctx) return 0;
    int64_t n;
    {
        std::lock_guard<std::mutex> lk(ctx->mu);
        n = (int64_t)ctx->gpu.device_bytes();
    }
    for (jp2hip_ctx *p : ctx->peers) n += jp2hip_device_bytes(p);
    return n;
}

int jp2hip_set_memory_limits(jp2hip_ctx *ctx, int64_t soft, int64_t hard) {
    if (!ctx) return fail("null context");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->mem_soft = soft > 0 ? soft : 0;
    ctx->gpu.set_limits(ctx->gpu.soft_limit(), hard > 0 ? (size_t)hard : SIZE_MAX);
    for (jp2hip_ctx *p : ctx->peers)
        if (jp2hip_set_memory_limits(p, soft, hard) != 0) return -1;
    return 0;
}

const char *jp2hip_dma_engines(void) {
    thread_local std::string s;
    s = jp2hip::dma_engine_report();
    return s.c_str();
}

int jp2hip_device_memory(int device, int64_t *free_bytes, int64_t *total_bytes) {
    int prev = -1;
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (hipSetDevice(device) != hipSuccess) return fail("device ordinal " + std::to_string(device) + " not usable");
    size_t fr = 0, tot = 0;
    const hipError_t e = hipMemGetInfo(&fr, &tot);
    if (prev >= 0) (void)hipSetDevice(prev);
    if (e != hipSuccess) return fail(std::string("hipMemGetInfo: ") + hipGetErrorString(e));
    if (free_bytes) *free_bytes = (int64_t)fr;
    if (total_bytes) *total_bytes = (int64_t)tot;
    return 0;
}

void jp2hip_destroy(jp2hip_ctx *ctx) {
    if (!ctx) return;
    {
        std::lock_guard<std::mutex> lk(g_reg_mu);
        g_reg.erase(std::remove(g_reg.begin(), g_reg.end(), ctx), g_reg.end());
    }
    g_live_contexts--;  // its peers count themselves down as they go
    delete ctx;
}

int jp2hip_tiff_layout(const uint8_t *tiff, size_t len, jp2hip_layout *layout, uint64_t *offsets,
                       int32_t max_offsets) {
    if (!layout) return fail("null layout");
    std::vector<uint64_t> offs;
    if (parse_tiff(tiff, len, layout, offs)) return -1;
    if ((int32_t)offs.size() > max_offsets || !offsets) {
        layout->strip_offsets = nullptr;
        return fail("offsets array too small: need " + std::to_string(offs.size()));
    }
    std::memcpy(offsets, offs.data(), offs.size() * sizeof(uint64_t));
    layout->strip_offsets = offsets;
    layout->strip_bytes = (layout->compression > 1 || layout->tile_width > 0) ? offsets + layout->nstrips : nullptr;
    return 0;
}

int jp2hip_encode_device(jp2hip_ctx *ctx, const void *d_src, size_t src_len, const jp2hip_layout *layout,
                         int conversion, const jp2hip_recipe *recipe, uint8_t **out, size_t *out_len,
                         jp2hip_stats *stats) {
    if (!ctx || !out || !out_len) return fail("null argument");
    *out = nullptr;
    *out_len = 0;
    double t0 = now_ms();
    std::lock_guard<std::mutex> lk(ctx->mu);
    return encode_core(ctx, d_src, src_len, layout, conversion, recipe, out, out_len, stats, t0, 0.0);
}

int jp2hip_encode_tiff(jp2hip_ctx *ctx, const uint8_t *tiff, size_t len, int conversion,
                       const jp2hip_recipe *recipe, uint8_t **out, size_t *out_len, jp2hip_stats *stats) {
    if (!ctx || !out || !out_len) return fail("null argument");
    *out = nullptr;
    *out_len = 0;
    double t0 = now_ms();
    jp2hip_layout lay;
    std::vector<uint64_t> offs;
    if (parse_tiff(tiff, len, &lay, offs)) return -1;
    if (wants_split(ctx, lay))
        return encode_split_host(ctx, tiff, len, lay, conversion, recipe, -1, out, out_len, stats, t0);
    std::lock_guard<std::mutex> lk(ctx->mu);
    std::string err;
    double th = now_ms();
    if (!ctx->gpu.upload_source(tiff, len, err)) return fail(err);
    double h2d = now_ms() - th;
    return encode_core(ctx, ctx->gpu.source(), len, &lay, conversion, recipe, out, out_len, stats, t0, h2d);
}

int jp2hip_encode_file(jp2hip_ctx *ctx, const char *tiff_path, const char *out_path, int conversion,
                       const jp2hip_recipe *recipe, jp2hip_stats *stats) {
    if (!ctx || !tiff_path || !out_path) return fail("null argument");
    const double t0 = now_ms();
    MappedFile mf;
    if (!mf.open(tiff_path)) {
        if (mf.fd < 0) return fail(std::string("cannot open TIFF: ") + tiff_path);
        return fail(std::string("cannot read TIFF: ") + tiff_path);
    }
    jp2hip_layout lay;
    std::vector<uint64_t> offs;
    if (parse_tiff(mf.p, mf.n, &lay, offs)) return -1;
    const std::string tmp = temp_name(out_path);
    if (wants_split(ctx, lay)) {
        // every rank writes its part at its offset of the temp file
        const int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
        if (fd < 0) return fail(std::string("cannot write output: ") + out_path);
        const int rc = encode_split_host(ctx, mf.p, mf.n, lay, conversion, recipe, fd, nullptr, nullptr, stats, t0);
        const bool closed = ::close(fd) == 0;
        if (rc != 0 || !closed || std::rename(tmp.c_str(), out_path) != 0) {
            std::remove(tmp.c_str());
            return rc != 0 ? -1 : fail(std::string("cannot write output: ") + out_path);
        }
        return 0;
    }
    uint8_t *out = nullptr;
    size_t olen = 0;
    if (jp2hip_encode_tiff(ctx, mf.p, mf.n, conversion, recipe, &out, &olen, stats)) return -1;
    FILE *o = std::fopen(tmp.c_str(), "wb");
    if (!o) {
        out_free(out);
        return fail(std::string("cannot write output: ") + out_path);
    }
    bool ok = std::fwrite(out, 1, olen, o) == olen;
    ok = (std::fclose(o) == 0) && ok;
    out_free(out);
    if (!ok || std::rename(tmp.c_str(), out_path) != 0) {
        std::remove(tmp.c_str());
        return fail(std::string("cannot write output: ") + out_path);
    }
    if (stats) stats->total_ms = now_ms() - t0;
    return 0;
}

int64_t jp2hip_tiff_pixels(const char *tiff_path) {
    if (!tiff_path) return fail("null argument");
    MappedFile mf;
    if (!mf.open(tiff_path)) return fail(std::string("cannot open TIFF: ") + tiff_path);
    jp2hip_layout lay;
    std::vector<uint64_t> offs;
    if (parse_tiff(mf.p, mf.n, &lay, offs)) return -1;
    return (int64_t)lay.width * lay.height;
}

int jp2hip_split_peers(jp2hip_ctx *ctx, const int32_t *ordinals, int32_t n, int64_t min_pixels) {
    if (!ctx || n < 0 || (n > 0 && !ordinals)) return fail("null argument");
    if (n > 64) return fail("split: at most 64 peers");
    std::lock_guard<std::mutex> lk(ctx->mu);
    std::vector<jp2hip_ctx *> made;
    for (int i = 0; i < n; i++) {
        jp2hip_config c = ctx->cfg;
        c.device = ordinals[i];
        jp2hip_ctx *p = nullptr;
        if (jp2hip_create(&p, &c) != 0) {
            const std::string e = std::string("split peer on device ") + std::to_string(ordinals[i]) + ": " + g_err;
            for (jp2hip_ctx *q : made) jp2hip_destroy(q);
            return fail(e);
        }
        made.push_back(p);
    }
    for (jp2hip_ctx *p : ctx->peers) jp2hip_destroy(p);
    ctx->peers = made;
    ctx->split_min_pixels = std::max<int64_t>(0, min_pixels);
    return 0;
}

int jp2hip_encode_device_split(jp2hip_ctx *ctx, const void *d_src, size_t src_len, const jp2hip_layout *layout,
                               int conversion, const jp2hip_recipe *recipe, const jp2hip_split *split,
                               uint8_t **out, size_t *out_len, uint64_t *file_offset, uint64_t *file_len,
                               jp2hip_stats *stats) {
    if (!ctx || !out || !out_len) return fail("null argument");
    *out = nullptr;
    *out_len = 0;
    double t0 = now_ms();
    std::lock_guard<std::mutex> lk(ctx->mu);
    return encode_split_core(ctx, d_src, src_len, layout, conversion, recipe, split, out, out_len, file_offset,
                             file_len, stats, t0);
}

void jp2hip_free(void *p) { out_free(p); }

}  // extern "C"
