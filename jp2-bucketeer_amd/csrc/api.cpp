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
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <unistd.h>

#include "gpu_encoder.h"
#include "jp2hip.h"
#include "jp2hip_internal.h"

struct jp2hip_ctx {
    std::mutex mu;
    jp2hip::GpuEncoder gpu;
    jp2hip_config cfg;
    int threads = 1;
    jp2hip::T2State t2;  // tier-2 arenas, reused call to call
};

namespace {

thread_local std::string g_err;

int fail(const std::string &msg) {
    g_err = msg;
    return -1;
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
            if (offs[s] + nb > len) return fail("tiff: strip " + std::to_string(s) + " out of range");
            const uint64_t unit = (uint64_t)tw * (planar == 2 ? 1 : spp) * (bps / 8) * th;
            if (tiled && comp == 1 && nb < unit) return fail("tiff: tile byte count too small");
            offs[need + s] = nb;
            continue;
        }
        if (offs[s] + row * rows > len) return fail("tiff: strip " + std::to_string(s) + " out of range");
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
}

// Slope prediction's rate target (bytes; 0 = prediction off) -- the same
// floor(rate * W * H / 8) the oracle's predict_and_code uses.
int64_t skip_target_of(const jp2hip_recipe &rc, int w, int h) {
    if (!rc.slope_skip || rc.rate_bpp <= 0.0) return 0;
    return (int64_t)std::floor(rc.rate_bpp * (double)w * (double)h / 8.0);
}

// Safety net of the prediction (oracle predict_and_code): planes were
// skipped, yet all coded bytes together stay below the target.
void undershoot_terms(const jp2hip::GpuEncoder &g, int64_t &coded, int64_t &skipped) {
    coded = 0;
    skipped = 0;
    const std::vector<int32_t> &len = g.block_lengths();
    const std::vector<uint8_t> &pm = g.block_pmin();
    for (size_t b = 0; b < len.size(); b++) coded += len[b];
    for (size_t b = 0; b < pm.size(); b++) skipped |= pm[b] > 0;
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

// The whole encode with the source already in device memory.  On success
// *out is a malloc'd buffer holding the complete file.
int encode_core(jp2hip_ctx *ctx, const void *d_src, size_t src_len, const jp2hip_layout *lay,
                int conversion, const jp2hip_recipe *recipe, uint8_t **out, size_t *out_len,
                jp2hip_stats *stats, double t_start, double h2d_ms) {
    using namespace jp2hip;
    if (conversion != JP2HIP_LOSSY && conversion != JP2HIP_LOSSLESS)
        return fail("conversion must be JP2HIP_LOSSY (0) or JP2HIP_LOSSLESS (1)");
    jp2hip_recipe rc;
    if (recipe) rc = *recipe;
    else default_recipe(&rc, conversion);
    if (!lay || !d_src) return fail("null source or layout");
    Plan plan;
    std::string err;
    jp2hip_layout ulay;
    std::vector<uint64_t> uoffs;
    if (!unpack_if_compressed(ctx, d_src, src_len, lay, ulay, uoffs, err)) return fail(err);
    if (!build_plan(plan, rc, lay->width, lay->height, lay->components, lay->bits, err)) return fail(err);
    const bool prof = ctx->cfg.profile != 0;
    StageTimes st;
    const int64_t skip_target = skip_target_of(rc, plan.w, plan.h);
    if (!ctx->gpu.run_front(d_src, *lay, plan, prof, st, err, skip_target)) return fail(err);
    if (skip_target > 0) {
        int64_t coded, skipped;
        undershoot_terms(ctx->gpu, coded, skipped);
        if (skipped && coded < skip_target && !ctx->gpu.run_front(d_src, *lay, plan, prof, st, err, 0))
            return fail(err);
    }
    const int nb = (int)plan.blocks.size();
    const int L = rc.layers;
    const std::vector<int32_t> &len = ctx->gpu.block_lengths();
    std::vector<uint8_t> h_nl;
    std::vector<int32_t> h_lrate;
    std::vector<int64_t> budgets((size_t)L, 0);
    T2Input in;
    in.plan = &plan;
    in.P = ctx->gpu.block_planes().data();
    in.data = nullptr;
    in.data_off = nullptr;
    in.threads = ctx->threads;
    T2State &t2 = ctx->t2;
    double t2ms = 0;
    int iters = 0;
    int64_t cs_bytes = 0;
    if (rc.rate_bpp <= 0.0) {
        // lossless: layer l keeps every pass whose slope clears total >> (L-1-l)
        int64_t total = 0;
        for (int b = 0; b < nb; b++) total += len[b];
        for (int l = 0; l < L; l++) budgets[l] = total >> (L - 1 - l);
        if (!ctx->gpu.select(plan, budgets, h_nl, h_lrate, prof, st, err)) return fail(err);
        iters = 1;
        in.nl = h_nl.data();
        in.lrate = h_lrate.data();
        const double t0 = now_ms();
        cs_bytes = t2_headers(in, t2);
        t2ms += now_ms() - t0;
    } else {
        const int64_t target = (int64_t)std::floor(rc.rate_bpp * (double)plan.w * (double)plan.h / 8.0);
        int64_t budget = target - 12 * plan.npackets - 16 * plan.ntileparts - 256;
        for (int it = 0; it < 8; it++) {
            if (budget < 0) budget = 0;
            for (int l = 0; l < L; l++) budgets[l] = budget >> (L - 1 - l);
            if (!ctx->gpu.select(plan, budgets, h_nl, h_lrate, prof, st, err)) return fail(err);
            iters++;
            in.nl = h_nl.data();
            in.lrate = h_lrate.data();
            const double t0 = now_ms();
            cs_bytes = t2_headers(in, t2);
            t2ms += now_ms() - t0;
            if (cs_bytes <= target) break;
            // exponential back-off + 1/16 of the overshoot + 64 B, as the oracle
            budget -= ((cs_bytes - target) << it) + ((cs_bytes - target) >> 4) + 64;
        }
    }
    // t2 now describes the final layer table; fetch the bytes it includes
    std::vector<int32_t> final_len((size_t)nb);
    std::vector<uint64_t> offs((size_t)nb);
    uint64_t total = 0;
    for (int b = 0; b < nb; b++) {
        final_len[b] = h_lrate[(size_t)b * L + (L - 1)];
        offs[b] = total;
        total += (uint64_t)final_len[b];
    }
    const uint8_t *data = nullptr;
    const double tg = now_ms();
    if (!ctx->gpu.gather(plan, final_len, offs, total, &data, prof, st, err)) return fail(err);
    const double gather_ms = now_ms() - tg;
    in.data = data;
    in.data_off = offs.data();
    const double t0 = now_ms();
    const size_t fh = file_header_bytes(plan);
    const size_t n = fh + (size_t)cs_bytes;
    uint8_t *buf = (uint8_t *)std::malloc(n);
    if (!buf) return fail("out of memory");
    write_file_header(plan, (uint64_t)cs_bytes, buf);
    t2_emit(in, t2, buf + fh);
    t2ms += now_ms() - t0;
    *out = buf;
    *out_len = n;
    if (stats) {
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
        stats->d2h_ms = prof ? st.d2h : gather_ms;
        stats->t2_ms = t2ms;
        stats->codeblocks = nb;
        int64_t tb = 0, tp = 0;
        ctx->gpu.t1_total_bytes(tb, tp);
        stats->t1_bytes = tb;
        stats->coded_passes = tp;
        stats->out_bytes = (int64_t)n;
        stats->rate_iterations = iters;
    }
    return 0;
}

// Tile-split encode (jp2hip.h, jp2hip_encode_device_split; split.cpp has the
// exchange rule).  Rank `rank` runs the device pipeline on its band of tile
// rows only; budgets, thresholds and tier-2 sizes are agreed through
// sp->allreduce_sum so the parts concatenate to the single-GPU file.
int encode_split_core(jp2hip_ctx *ctx, const void *d_src, const jp2hip_layout *lay, int conversion,
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
    jp2hip_recipe rc;
    if (recipe) rc = *recipe;
    else default_recipe(&rc, conversion);
    if (!lay || !d_src) return fail("null source or layout");
    Plan full;
    std::string err;
    // every rank sees the same layout, so all of them stop here together
    if (lay->compression > 1 || lay->tile_width > 0)
        return fail("split: compressed or tiled TIFFs are not supported; rewrite as uncompressed strips first");
    if (!build_plan(full, rc, lay->width, lay->height, lay->components, lay->bits, err)) return fail(err);
    int tr0, tr1;
    split_tile_rows(full.nty, rank, world, tr0, tr1);
    Plan sub;
    make_subplan(full, tr0, tr1, sub);
    const bool have = sub.ntc > 0;
    const bool prof = ctx->cfg.profile != 0;
    StageTimes st;
    std::vector<uint64_t> keys;
    std::vector<int64_t> cum;
    // slope prediction over the whole image: the plane histogram is summed
    // over ranks (one all-reduce of kSlopeBins + 1 int64, the last entry a
    // failure flag, so a rank that failed earlier still joins the exchange)
    const int64_t skip_target = skip_target_of(rc, full.w, full.h);
    bool hist_done = false;
    GpuEncoder::HistReduce reduce = [&](std::vector<int64_t> &h) {
        hist_done = true;
        std::vector<int64_t> v(h.size() + 1, 0);
        std::copy(h.begin(), h.end(), v.begin());
        if (!allreduce(v.data(), (int)v.size()) || v.back() != 0) return false;
        std::copy(v.begin(), v.end() - 1, h.begin());
        return true;
    };
    bool ok = !have || ctx->gpu.run_front(d_src, *lay, sub, prof, st, err, skip_target, &reduce);
    if (skip_target > 0 && !hist_done) {  // no blocks here, or failed before the exchange
        std::vector<int64_t> v((size_t)kSlopeBins + 1, 0);
        v.back() = ok ? 0 : 1;
        if (!allreduce(v.data(), (int)v.size())) return fail("split: all-reduce failed");
        if (ok && v.back()) { ok = false; err = "split: another rank failed"; }
    }
    if (skip_target > 0) {  // the prediction's safety net, decided globally
        int64_t v[3] = {0, 0, ok ? 0 : 1};
        if (ok && have) undershoot_terms(ctx->gpu, v[0], v[1]);
        if (!allreduce(v, 3)) return fail("split: all-reduce failed");
        if (ok && v[2]) { ok = false; err = "split: another rank failed"; }
        if (ok && v[1] && v[0] < skip_target && have)
            ok = ctx->gpu.run_front(d_src, *lay, sub, prof, st, err, 0);
    }
    ok = ok && (!have || ctx->gpu.segments(keys, cum, err));
    {
        int64_t flag = ok ? 0 : 1;
        if (!allreduce(&flag, 1)) return fail("split: all-reduce failed");
        if (!ok) return fail(err);
        if (flag) return fail("split: another rank failed");
    }
    const int L = rc.layers;
    const size_t nbf = full.blocks.size(), nbl = sub.blocks.size(), b0 = (size_t)sub.block0;
    std::vector<uint8_t> P_full(nbf, 0), nl_full(nbf * L, 0), h_nl;
    std::vector<int32_t> lrate_full(nbf * L, 0), h_lrate;
    if (have) std::copy(ctx->gpu.block_planes().begin(), ctx->gpu.block_planes().begin() + nbl, P_full.begin() + b0);
    T2Input in;
    in.plan = &full;
    in.P = P_full.data();
    in.nl = nl_full.data();
    in.lrate = lrate_full.data();
    in.data = nullptr;
    in.data_off = nullptr;
    in.threads = ctx->threads;
    in.tile0 = sub.tile0;
    in.tile1 = sub.tile0 + full.ntx * (tr1 - tr0);
    T2State &t2 = ctx->t2;
    std::vector<int64_t> budgets((size_t)L, 0);
    std::vector<uint64_t> K((size_t)L);
    double t2ms = 0;
    int iters = 0;
    int64_t cs_bytes = 0;
    // one selection + header pass for `budgets`; returns false on failure
    auto round = [&]() -> bool {
        if (jp2hip_split_thresholds(keys.data(), cum.data(), (int64_t)keys.size(), budgets.data(), L, sp,
                                    K.data()) != 0) {
            err = "split: threshold exchange failed";
            return false;
        }
        bool rok = true;
        if (have) {
            rok = ctx->gpu.select_keys(sub, K, h_nl, h_lrate, prof, st, err);
            if (rok) {
                std::copy(h_nl.begin(), h_nl.end(), nl_full.begin() + b0 * L);
                std::copy(h_lrate.begin(), h_lrate.end(), lrate_full.begin() + b0 * L);
            }
        }
        const double t0 = now_ms();
        int64_t v[2] = {0, rok ? 0 : 1};
        if (rok) v[0] = t2_headers(in, t2) - (int64_t)t2.main.size() - 2;
        t2ms += now_ms() - t0;
        if (!allreduce(v, 2)) { err = "split: all-reduce failed"; return false; }
        if (v[1]) { if (rok) err = "split: another rank failed"; return false; }
        cs_bytes = (int64_t)t2.main.size() + 2 + v[0];
        iters++;
        return true;
    };
    if (rc.rate_bpp <= 0.0) {
        int64_t total = 0;
        if (have)
            for (size_t b = 0; b < nbl; b++) total += ctx->gpu.block_lengths()[b];
        if (!allreduce(&total, 1)) return fail("split: all-reduce failed");
        for (int l = 0; l < L; l++) budgets[l] = total >> (L - 1 - l);
        if (!round()) return fail(err);
    } else {
        const int64_t target = (int64_t)std::floor(rc.rate_bpp * (double)full.w * (double)full.h / 8.0);
        int64_t budget = target - 12 * full.npackets - 16 * full.ntileparts - 256;
        for (int it = 0; it < 8; it++) {
            if (budget < 0) budget = 0;
            for (int l = 0; l < L; l++) budgets[l] = budget >> (L - 1 - l);
            if (!round()) return fail(err);
            if (cs_bytes <= target) break;
            budget -= ((cs_bytes - target) << it) + ((cs_bytes - target) >> 4) + 64;  // as encode_core
        }
    }
    // this rank's included bytes
    std::vector<int32_t> final_len(nbl);
    std::vector<uint64_t> offs(nbl), offs_full(nbf, 0);
    uint64_t total = 0;
    for (size_t b = 0; b < nbl; b++) {
        final_len[b] = h_lrate[b * L + (L - 1)];
        offs[b] = total;
        offs_full[b0 + b] = total;
        total += (uint64_t)final_len[b];
    }
    const uint8_t *data = nullptr;
    const double tg = now_ms();
    ok = !have || ctx->gpu.gather(sub, final_len, offs, total, &data, prof, st, err);
    const double gather_ms = now_ms() - tg;
    const bool with_main = rank == 0, with_eoc = rank == world - 1;
    const size_t fh = with_main ? file_header_bytes(full) : 0;
    const uint64_t part = ok ? fh + t2_part_bytes(in, t2, with_main, with_eoc) : 0;
    std::vector<int64_t> sizes((size_t)world + 1, 0);
    sizes[rank] = (int64_t)part;
    sizes[world] = ok ? 0 : 1;
    if (!allreduce(sizes.data(), world + 1)) return fail("split: all-reduce failed");
    if (!ok) return fail(err);
    if (sizes[world]) return fail("split: another rank failed");
    uint64_t off = 0, flen = 0;
    for (int r = 0; r < world; r++) {
        if (r < rank) off += (uint64_t)sizes[r];
        flen += (uint64_t)sizes[r];
    }
    in.data = data;
    in.data_off = offs_full.data();
    const double t0 = now_ms();
    uint8_t *buf = (uint8_t *)std::malloc(part ? part : 1);
    if (!buf) return fail("out of memory");
    if (with_main) write_file_header(full, (uint64_t)cs_bytes, buf);
    t2_emit_part(in, t2, buf + fh, with_main, with_eoc);
    t2ms += now_ms() - t0;
    *out = buf;
    *out_len = part;
    if (file_offset) *file_offset = off;
    if (file_len) *file_len = flen;
    if (stats) {
        std::memset(stats, 0, sizeof *stats);
        stats->total_ms = now_ms() - t_start;
        stats->ingest_ms = st.ingest;
        stats->dwt_ms = st.dwt;
        stats->quant_ms = st.quant;
        stats->t1_ms = st.t1_cm + st.t1_mq;
        stats->t1_cm_ms = st.t1_cm;
        stats->t1_mq_ms = st.t1_mq;
        stats->pcrd_ms = st.pcrd;
        stats->d2h_ms = prof ? st.d2h : gather_ms;
        stats->t2_ms = t2ms;
        stats->codeblocks = (int64_t)nbl;
        if (have) {
            int64_t tb = 0, tp = 0;
            ctx->gpu.t1_total_bytes(tb, tp);
            stats->t1_bytes = tb;
            stats->coded_passes = tp;
        }
        stats->out_bytes = (int64_t)flen;
        stats->rate_iterations = iters;
    }
    return 0;
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

void jp2hip_recipe_init(jp2hip_recipe *recipe, int conversion) {
    if (recipe) default_recipe(recipe, conversion);
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
        return fail("device ordinal out of range");
    }
    std::string err;
    if (!c->gpu.init(c->cfg.device, err)) {
        delete c;
        return fail(err);
    }
    *out = c;
    return 0;
}

void jp2hip_destroy(jp2hip_ctx *ctx) { delete ctx; }

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
    FILE *f = std::fopen(tiff_path, "rb");
    if (!f) return fail(std::string("cannot open TIFF: ") + tiff_path);
    std::vector<uint8_t> buf;
    if (std::fseek(f, 0, SEEK_END) == 0) {
        long n = std::ftell(f);
        if (n > 0) {
            buf.resize((size_t)n);
            std::fseek(f, 0, SEEK_SET);
            if (std::fread(buf.data(), 1, buf.size(), f) != buf.size()) buf.clear();
        }
    }
    std::fclose(f);
    if (buf.empty()) return fail(std::string("cannot read TIFF: ") + tiff_path);
    uint8_t *out = nullptr;
    size_t olen = 0;
    if (jp2hip_encode_tiff(ctx, buf.data(), buf.size(), conversion, recipe, &out, &olen, stats)) return -1;
    std::string tmp = std::string(out_path) + ".part-" + std::to_string((long)getpid()) + "-" +
                      std::to_string((unsigned long)std::hash<std::thread::id>()(std::this_thread::get_id()) % 100000);
    FILE *o = std::fopen(tmp.c_str(), "wb");
    if (!o) {
        std::free(out);
        return fail(std::string("cannot write output: ") + out_path);
    }
    bool ok = std::fwrite(out, 1, olen, o) == olen;
    ok = (std::fclose(o) == 0) && ok;
    std::free(out);
    if (!ok || std::rename(tmp.c_str(), out_path) != 0) {
        std::remove(tmp.c_str());
        return fail(std::string("cannot write output: ") + out_path);
    }
    return 0;
}

int jp2hip_encode_device_split(jp2hip_ctx *ctx, const void *d_src, size_t src_len, const jp2hip_layout *layout,
                               int conversion, const jp2hip_recipe *recipe, const jp2hip_split *split,
                               uint8_t **out, size_t *out_len, uint64_t *file_offset, uint64_t *file_len,
                               jp2hip_stats *stats) {
    if (!ctx || !out || !out_len) return fail("null argument");
    *out = nullptr;
    *out_len = 0;
    (void)src_len;
    double t0 = now_ms();
    std::lock_guard<std::mutex> lk(ctx->mu);
    return encode_split_core(ctx, d_src, layout, conversion, recipe, split, out, out_len, file_offset, file_len,
                             stats, t0);
}

void jp2hip_free(void *p) { std::free(p); }

}  // extern "C"
