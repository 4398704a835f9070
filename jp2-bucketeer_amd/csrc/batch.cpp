// batch.cpp -- the batch path (include/jp2hip.h, "Batch path"): one GPU's
// work queue for a CSV batch.
//
// Reference chain it replaces, per CSV row (src/main/java/edu/ucla/library/
// bucketeer/...): handlers/LoadCsvHandler.java:250-289 queues the rows ->
// verticles/LargeImageVerticle.java:65-108 posts each to loadImage ->
// verticles/ImageWorkerVerticle.java:54-110 converts (Conversion.LOSSLESS),
// replies, then sends the JPX to verticles/S3BucketVerticle.java:88-211 with
// derivative-image=true, which deletes it after the upload (:286-303).  There
// the whole chain runs on one worker thread per instance, serially
// (MainVerticle.java:229-231).
//
// Here, per GPU:
//   readers    TIFF file -> pinned host buffer (reused pool), header parse
//   encoders   one per context: jp2hip_encode_tiff on the context's own HIP
//              stream (H2D, device pipeline, tier-2), so `contexts` images are
//              in flight on the GPU and one image's tier-2 overlaps another's
//              kernels
//   uploaders  atomic JPX write (temp + rename), upload hook, delete
// Bounded queues between the stages keep at most contexts + readers images
// in host memory.  Failures never stop the batch: each job ends in exactly
// one result with its status (ImageWorker's reply / callback "true|false").
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <unistd.h>

#include "jp2hip.h"

namespace {

double now_ms() {
    using namespace std::chrono;
    return duration<double, std::milli>(steady_clock::now().time_since_epoch()).count();
}

template <typename T>
class Queue {
  public:
    explicit Queue(size_t cap) : cap_(cap) {}
    void set_capacity(size_t cap) { cap_ = cap; }  // before any producer runs
    // false once closed
    bool push(T &&v) {
        std::unique_lock<std::mutex> lk(mu_);
        not_full_.wait(lk, [&] { return closed_ || q_.size() < cap_; });
        if (closed_) return false;
        q_.push_back(std::move(v));
        not_empty_.notify_one();
        return true;
    }
    // false once closed and drained
    bool pop(T &out) {
        std::unique_lock<std::mutex> lk(mu_);
        not_empty_.wait(lk, [&] { return closed_ || !q_.empty(); });
        if (q_.empty()) return false;
        out = std::move(q_.front());
        q_.pop_front();
        not_full_.notify_one();
        return true;
    }
    void close() {
        std::lock_guard<std::mutex> lk(mu_);
        closed_ = true;
        not_empty_.notify_all();
        not_full_.notify_all();
    }

  private:
    size_t cap_;
    bool closed_ = false;
    std::deque<T> q_;
    std::mutex mu_;
    std::condition_variable not_empty_, not_full_;
};

struct Job {
    int64_t job = 0;
    std::string id, tiff, jpx;
    int conversion = JP2HIP_LOSSLESS;
    bool has_recipe = false;
    jp2hip_recipe recipe;
    // filled along the pipeline
    uint8_t *src = nullptr;  // pinned TIFF bytes
    size_t src_cap = 0, src_len = 0;
    uint8_t *jpx_bytes = nullptr;  // malloc'd by jp2hip_encode_tiff
    size_t jpx_len = 0;
    jp2hip_batch_result res;
};

void set_msg(jp2hip_batch_result &r, const std::string &m) {
    std::snprintf(r.message, sizeof r.message, "%s", m.c_str());
}

// built-in upload stub: read every byte back (FakeS3BucketVerticle replies
// success without looking; reading keeps the I/O honest)
int stub_upload(void *, const char *, const char *path) {
    FILE *f = std::fopen(path, "rb");
    if (!f) return -1;
    std::vector<uint8_t> buf(1 << 20);
    uint64_t sum = 0;
    size_t n;
    while ((n = std::fread(buf.data(), 1, buf.size(), f)) > 0)
        for (size_t i = 0; i < n; i += 4096) sum += buf[i];
    std::fclose(f);
    (void)sum;
    return 0;
}

}  // namespace

struct jp2hip_batch {
    jp2hip_batch_config cfg;
    jp2hip_upload_fn upload = nullptr;
    void *user = nullptr;
    std::vector<jp2hip_ctx *> ctxs;
    Queue<Job> submitted{(size_t)1 << 40}, loaded{1}, encoded{1};
    std::vector<std::thread> readers, encoders, uploaders;
    // pinned buffer pool (readers take, encoders return)
    std::mutex pool_mu;
    std::vector<std::pair<uint8_t *, size_t>> pool;
    // results
    std::mutex res_mu;
    std::condition_variable res_cv;
    std::deque<jp2hip_batch_result> results;
    std::atomic<int64_t> pending{0};
    std::atomic<bool> closed{false};
    std::atomic<int> readers_left{0}, encoders_left{0};

    void finish(Job &j) {
        if (j.src) give_back(j.src, j.src_cap);
        j.src = nullptr;
        if (j.jpx_bytes) jp2hip_free(j.jpx_bytes);
        j.jpx_bytes = nullptr;
        {
            std::lock_guard<std::mutex> lk(res_mu);
            results.push_back(j.res);
        }
        res_cv.notify_all();
    }
    uint8_t *take(size_t n, size_t &cap) {
        {
            std::lock_guard<std::mutex> lk(pool_mu);
            for (size_t i = 0; i < pool.size(); i++)
                if (pool[i].second >= n) {
                    uint8_t *p = pool[i].first;
                    cap = pool[i].second;
                    pool.erase(pool.begin() + (long)i);
                    return p;
                }
        }
        void *p = nullptr;
        cap = n + n / 8 + 4096;
        if (hipHostMalloc(&p, cap, hipHostMallocDefault) != hipSuccess) {
            p = nullptr;
            cap = 0;
        }
        return (uint8_t *)p;
    }
    void give_back(uint8_t *p, size_t cap) {
        std::lock_guard<std::mutex> lk(pool_mu);
        pool.emplace_back(p, cap);
    }

    void reader() {
        Job j;
        std::vector<uint64_t> offs;
        while (submitted.pop(j)) {
            const double t0 = now_ms();
            FILE *f = std::fopen(j.tiff.c_str(), "rb");
            long n = -1;
            if (f && std::fseek(f, 0, SEEK_END) == 0) n = std::ftell(f);
            if (!f || n <= 0) {
                if (f) std::fclose(f);
                j.res.status = JP2HIP_BATCH_CONVERT_FAILED;
                set_msg(j.res, "cannot read TIFF: " + j.tiff);
                finish(j);
                continue;
            }
            j.src = take((size_t)n, j.src_cap);
            bool ok = j.src != nullptr && std::fseek(f, 0, SEEK_SET) == 0 &&
                      std::fread(j.src, 1, (size_t)n, f) == (size_t)n;
            std::fclose(f);
            if (!ok) {
                j.res.status = JP2HIP_BATCH_CONVERT_FAILED;
                set_msg(j.res, "cannot read TIFF: " + j.tiff);
                finish(j);
                continue;
            }
            j.src_len = (size_t)n;
            j.res.in_bytes = n;
            jp2hip_layout lay;
            std::memset(&lay, 0, sizeof lay);
            if (offs.size() < 1024) offs.resize(1024);
            int prc = jp2hip_tiff_layout(j.src, j.src_len, &lay, offs.data(), (int32_t)offs.size());
            // more strips / tiles than slots: the parse already counted them
            // (offsets + byte counts for compressed or tiled files)
            if (prc != 0 && lay.nstrips > 0 && 2 * (size_t)lay.nstrips > offs.size()) {
                offs.resize(2 * (size_t)lay.nstrips);
                prc = jp2hip_tiff_layout(j.src, j.src_len, &lay, offs.data(), (int32_t)offs.size());
            }
            if (prc != 0) {
                j.res.status = JP2HIP_BATCH_CONVERT_FAILED;
                set_msg(j.res, std::string("Failed to convert TIFF to JP2: ") + j.id + ": " + jp2hip_last_error());
                finish(j);
                continue;
            }
            j.res.pixels = (int64_t)lay.width * lay.height;
            j.res.read_ms = now_ms() - t0;
            if (!loaded.push(std::move(j))) break;
        }
        if (--readers_left == 0) loaded.close();
    }

    void encoder(jp2hip_ctx *ctx) {
        Job j;
        while (loaded.pop(j)) {
            const double t0 = now_ms();
            jp2hip_stats st;
            const int rc = jp2hip_encode_tiff(ctx, j.src, j.src_len, j.conversion,
                                              j.has_recipe ? &j.recipe : nullptr, &j.jpx_bytes, &j.jpx_len, &st);
            give_back(j.src, j.src_cap);
            j.src = nullptr;
            j.res.encode_ms = now_ms() - t0;
            if (rc != 0) {
                j.res.status = JP2HIP_BATCH_CONVERT_FAILED;
                set_msg(j.res, std::string("Failed to convert TIFF to JP2: ") + j.id + ": " + jp2hip_last_error());
                finish(j);
                continue;
            }
            j.res.out_bytes = (int64_t)j.jpx_len;
            if (!encoded.push(std::move(j))) break;
        }
        if (--encoders_left == 0) encoded.close();
    }

    void uploader() {
        Job j;
        while (encoded.pop(j)) {
            const double t0 = now_ms();
            bool ok = true;
            std::string err;
            if (cfg.write_output) {
                const std::string tmp = j.jpx + ".part-" + std::to_string((long)getpid()) + "-" +
                                        std::to_string((long long)j.job);
                FILE *o = std::fopen(tmp.c_str(), "wb");
                ok = o != nullptr;
                if (ok) {
                    ok = std::fwrite(j.jpx_bytes, 1, j.jpx_len, o) == j.jpx_len;
                    ok = (std::fclose(o) == 0) && ok;
                }
                if (ok) ok = std::rename(tmp.c_str(), j.jpx.c_str()) == 0;
                if (!ok) {
                    std::remove(tmp.c_str());
                    j.res.status = JP2HIP_BATCH_CONVERT_FAILED;
                    set_msg(j.res, "cannot write output: " + j.jpx);
                } else {
                    const int u = (upload ? upload : stub_upload)(user, j.id.c_str(), j.jpx.c_str());
                    if (u != 0) {
                        j.res.status = JP2HIP_BATCH_UPLOAD_FAILED;
                        set_msg(j.res, "upload failed: " + j.id);
                    } else if (cfg.delete_after_upload) {
                        std::remove(j.jpx.c_str());
                    }
                }
            }
            j.res.upload_ms = now_ms() - t0;
            finish(j);
        }
    }
};

namespace {
thread_local std::string g_batch_err;
}

extern "C" {

int jp2hip_batch_create(jp2hip_batch **out, const jp2hip_batch_config *cfg, jp2hip_upload_fn upload, void *user) {
    if (!out) return -1;
    *out = nullptr;
    jp2hip_batch_config c;
    std::memset(&c, 0, sizeof c);
    if (cfg) c = *cfg;
    if (c.contexts <= 0) c.contexts = 12;  // ~12 images in flight per GPU
    if (c.reader_threads <= 0) c.reader_threads = 4;
    if (c.uploader_threads <= 0) c.uploader_threads = 4;
    if (c.host_threads <= 0) c.host_threads = std::max(2, 16 / c.contexts);
    jp2hip_batch *b = new jp2hip_batch();
    b->cfg = c;
    b->loaded.set_capacity((size_t)c.contexts);
    b->encoded.set_capacity((size_t)c.uploader_threads + 1);
    b->upload = upload;
    b->user = user;
    for (int i = 0; i < c.contexts; i++) {
        jp2hip_config cc;
        std::memset(&cc, 0, sizeof cc);
        cc.device = c.device;
        cc.host_threads = c.host_threads;
        jp2hip_ctx *ctx = nullptr;
        if (jp2hip_create(&ctx, &cc) != 0) {
            for (jp2hip_ctx *x : b->ctxs) jp2hip_destroy(x);
            delete b;
            return -1;  // jp2hip_last_error() holds the reason
        }
        b->ctxs.push_back(ctx);
    }
    b->readers_left = c.reader_threads;
    b->encoders_left = c.contexts;
    for (int i = 0; i < c.reader_threads; i++) b->readers.emplace_back([b] { b->reader(); });
    for (int i = 0; i < c.contexts; i++) b->encoders.emplace_back([b, i] { b->encoder(b->ctxs[i]); });
    for (int i = 0; i < c.uploader_threads; i++) b->uploaders.emplace_back([b] { b->uploader(); });
    *out = b;
    return 0;
}

int jp2hip_batch_submit(jp2hip_batch *b, int64_t job, const char *image_id, const char *tiff_path,
                        const char *jpx_path, int conversion, const jp2hip_recipe *recipe) {
    if (!b || !image_id || !tiff_path || !jpx_path || b->closed) return -1;
    Job j;
    j.job = job;
    j.id = image_id;
    j.tiff = tiff_path;
    j.jpx = jpx_path;
    j.conversion = conversion;
    if (recipe) {
        j.has_recipe = true;
        j.recipe = *recipe;
    }
    std::memset(&j.res, 0, sizeof j.res);
    j.res.job = job;
    b->pending++;
    if (!b->submitted.push(std::move(j))) {
        b->pending--;
        return -1;
    }
    return 0;
}

int jp2hip_batch_wait(jp2hip_batch *b, jp2hip_batch_result *results, int max, int timeout_ms) {
    if (!b || !results || max <= 0) return 0;
    std::unique_lock<std::mutex> lk(b->res_mu);
    auto ready = [&] { return !b->results.empty() || b->pending.load() == 0; };
    if (timeout_ms < 0) b->res_cv.wait(lk, ready);
    else b->res_cv.wait_for(lk, std::chrono::milliseconds(timeout_ms), ready);
    int n = 0;
    while (n < max && !b->results.empty()) {
        results[n++] = b->results.front();
        b->results.pop_front();
        b->pending--;
    }
    return n;
}

int64_t jp2hip_batch_pending(jp2hip_batch *b) { return b ? b->pending.load() : 0; }

void jp2hip_batch_destroy(jp2hip_batch *b) {
    if (!b) return;
    b->closed = true;
    b->submitted.close();
    for (auto &t : b->readers) t.join();
    for (auto &t : b->encoders) t.join();
    for (auto &t : b->uploaders) t.join();
    for (jp2hip_ctx *c : b->ctxs) jp2hip_destroy(c);
    for (auto &p : b->pool) (void)hipHostFree(p.first);
    delete b;
}

}  // extern "C"
