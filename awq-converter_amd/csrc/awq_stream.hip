// awq_stream.hip — the host streaming pipeline of include/awq_hip.h (awq_stream_*).
//
// Replaces the CLI's per-tensor loop (reference main.py:216-392: every file loaded whole,
// then tensor by tensor through the Python quantizer) with a native pipeline over batches
// of tensors that fill fixed staging slots:
//
//   reader threads   pread the batch's tensors from their files into pinned slot b % nslots
//                    (large tensors in 16 MiB pieces across the threads); a slot is refilled
//                    once the H2D copy of the batch that used it before has completed
//   submitter thread plans the batch's descriptors and tensor tables into the slot's table
//                    area (the first awq_stream_table_bytes of the slot), then ONE H2D of
//                    tables + input (h2d stream: no small table copies — those stalled the
//                    submitter for milliseconds, profiles/round3/r3m), then on the compute
//                    stream one ragged launch per dtype (awq_quantize_ragged) and
//                    awq_quantize_groups_ex for the shapes the ragged kernel does not take,
//                    then the D2H of the outputs of the tensors the batch completes (d2h
//                    stream, adjacent ranges coalesced)
//   caller           awq_stream_wait(b) per batch, then hands those tensors on (the CLI's
//                    chunk writer), while the next batches are read, copied and quantized.
//
// It is a client of the quantizer's own C ABI (awq_plan_ragged, awq_plan_block_tensor,
// awq_ragged_flags, awq_quantize_ragged, awq_quantize_groups_ex): the kernels see exactly the
// launches a single-process caller would make, on sub-tensors of whole rows.
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "awq_internal.h"

namespace {

constexpr int64_t kAlign = 256;             // slot offset of every piece (the kernels' 16-B loads)
constexpr int64_t kReadPiece = 16ll << 20;  // pread unit handed to one reader thread

int64_t elem_bytes(int dtype) { return dtype == AWQ_DTYPE_F64 ? 8 : (dtype == AWQ_DTYPE_F32 ? 4 : 2); }
int64_t align_up(int64_t v, int64_t a) { return (v + a - 1) / a * a; }
double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
bool aligned(const void* p, size_t a) { return ((uintptr_t)p % a) == 0; }

struct Piece {
    int item;
    int64_t row0, nrows;
    int64_t slot_off, bytes;
};

struct Batch {
    int slot;
    int64_t bytes;
    std::vector<Piece> pieces;
    int item_begin, item_end;   // the items whose last piece is in this batch
    int64_t dev_wait = -1;      // the batch whose D2H the kernels wait for (device ring reuse)
    int32_t host_gate = 0;      // releases the D2H waits for (host ring reuse)
};

struct ReadJob {
    int64_t batch;
    int piece;
    int64_t off, len;           // byte range inside the piece
};

struct Pipeline {
    std::vector<awq_stream_item> items;
    awq_stream_config cfg{};
    int device = 0;
    std::vector<Batch> batches;
    std::vector<ReadJob> jobs;
    std::vector<hipEvent_t> ev_h2d, ev_kern, ev_done;
    int64_t tb = 0, stride = 0;        // table area per slot; slot stride (tb + slot_bytes)
    hipEvent_t ev_start = nullptr;     // (trace only) the event clock's origin
    double ev_start_host = 0;          // (trace only) host clock (from t0) when it was recorded
    hipStream_t st_cs = nullptr, st_h2d = nullptr, st_d2h = nullptr;
    bool own_cs = false, own_h2d = false, own_d2h = false;   // created by the pipeline
    std::vector<double> tr;            // (trace only) AWQ_STREAM_TRACE_FIELDS per batch, host part
    std::mutex mu;
    std::condition_variable cv;
    std::vector<int64_t> reads_left;
    std::vector<int32_t> first_batch, last_batch;   // per item
    int64_t h2d_recorded = -1, done_recorded = -1;
    int32_t released = 0;              // awq_stream_release
    bool abort = false;                // awq_stream_end before the last batch was copied back
    size_t next_job = 0;
    int err = 0;
    std::string err_msg;
    std::vector<std::thread> readers;
    std::thread submitter;
    double t0 = 0, read_busy = 0, wait_read = 0, wait_slot = 0, wait_release = 0, prepare = 0;
    int64_t bytes_read = 0;

    void fail(int code, const std::string& msg) {
        std::lock_guard<std::mutex> g(mu);
        if (!err) {
            err = code;
            err_msg = msg;
        }
        cv.notify_all();
    }
    bool hip_ok(hipError_t e, const char* what) {
        if (e == hipSuccess) return true;
        fail(AWQ_EHIP, std::string(what) + ": " + hipGetErrorString(e));
        return false;
    }
};

// ---- planning ---------------------------------------------------------------------------
int plan(Pipeline& P, std::string& why) {
    const int64_t slot = P.cfg.slot_bytes;
    int64_t cap = P.cfg.first_batch_bytes > 0 ? std::min(P.cfg.first_batch_bytes, slot) : slot;
    Batch cur{0, 0, {}, 0, 0};
    auto close = [&](int item_end) {
        cur.item_end = item_end;
        P.batches.push_back(cur);
        cur = Batch{(int)(P.batches.size() % (size_t)P.cfg.nslots), 0, {}, item_end, item_end};
        cap = slot;
    };
    const int n = (int)P.items.size();
    for (int i = 0; i < n; ++i) {
        const awq_stream_item& it = P.items[i];
        const int64_t rowbytes = it.K * elem_bytes(it.dtype);
        int64_t r = 0;
        while (r < it.rows && rowbytes > 0) {
            const int64_t used = align_up(cur.bytes, kAlign);
            const int64_t avail = cap - used;
            const int64_t need = (it.rows - r) * rowbytes;
            const bool room = (int64_t)cur.pieces.size() < AWQ_STREAM_MAX_BATCH_ITEMS;
            int64_t take = 0;
            if (room && need <= avail) {
                take = it.rows - r;
            } else if (room && avail >= rowbytes) {
                take = avail / rowbytes;
                if (take >= 8) take -= take % 8;   // row splits on multiples of 8: aligned output rows
            }
            if (take == 0) {
                if (cur.pieces.empty()) {
                    why = "a row of " + std::to_string(rowbytes) + " B does not fit a staging slot of " +
                          std::to_string(slot) + " B";
                    return AWQ_EINVAL;
                }
                close(i);
                continue;
            }
            cur.pieces.push_back(Piece{i, r, take, used, take * rowbytes});
            cur.bytes = used + take * rowbytes;
            r += take;
        }
    }
    if (!cur.pieces.empty() || P.batches.empty() || cur.item_begin < n) close(n);
    // every item's first / last batch
    P.first_batch.assign(n, -1);
    P.last_batch.assign(n, -1);
    for (size_t b = 0; b < P.batches.size(); ++b) {
        const Batch& B = P.batches[b];
        for (const Piece& pc : B.pieces)
            if (P.first_batch[pc.item] < 0) P.first_batch[pc.item] = (int32_t)b;
        for (int i = B.item_begin; i < B.item_end; ++i) {
            P.last_batch[i] = (int32_t)b;
            if (P.first_batch[i] < 0) P.first_batch[i] = (int32_t)b;
        }
    }
    // ring gates: a batch's kernels wait for the D2H the device ranges they overwrite
    // needed; its D2H waits for the releases of the host ranges it overwrites
    for (int i = 0; i < n; ++i) {
        const awq_stream_item& it = P.items[i];
        if (it.dev_gate < 0 || it.dev_gate > i || it.host_gate < 0 || it.host_gate > i) {
            why = "item " + std::to_string(i) + ": a ring gate must name earlier items only";
            return AWQ_EINVAL;
        }
        if (it.dev_gate > 0) {
            const int32_t dep = P.last_batch[it.dev_gate - 1], at = P.first_batch[i];
            if (dep >= at) {
                why = "item " + std::to_string(i) + ": its device outputs overlap those of item " +
                      std::to_string(it.dev_gate - 1) + ", copied back in batch " + std::to_string(dep) +
                      ", not before its own kernels (batch " + std::to_string(at) + "): device output ring too small";
                return AWQ_EINVAL;
            }
            Batch& B = P.batches[at];
            B.dev_wait = std::max<int64_t>(B.dev_wait, dep);
        }
        Batch& L = P.batches[P.last_batch[i]];
        L.host_gate = std::max(L.host_gate, it.host_gate);
    }
    // reads: every piece in kReadPiece units, batch by batch
    P.reads_left.assign(P.batches.size(), 0);
    for (size_t b = 0; b < P.batches.size(); ++b) {
        const Batch& B = P.batches[b];
        for (size_t k = 0; k < B.pieces.size(); ++k)
            for (int64_t off = 0; off < B.pieces[k].bytes; off += kReadPiece) {
                P.jobs.push_back(ReadJob{(int64_t)b, (int)k, off, std::min(kReadPiece, B.pieces[k].bytes - off)});
                ++P.reads_left[b];
            }
    }
    return AWQ_OK;
}

// ---- reader threads ---------------------------------------------------------------------
void reader_main(Pipeline* P) {
    (void)hipSetDevice(P->device);
    for (;;) {
        ReadJob j;
        {
            std::lock_guard<std::mutex> g(P->mu);
            if (P->err || P->next_job >= P->jobs.size()) return;
            j = P->jobs[P->next_job++];
            if (!P->tr.empty() && P->tr[j.batch * AWQ_STREAM_TRACE_FIELDS] < 0)
                P->tr[j.batch * AWQ_STREAM_TRACE_FIELDS] = now_s() - P->t0;
        }
        const Batch& B = P->batches[j.batch];
        const int64_t prev = j.batch - P->cfg.nslots;   // the batch that used this slot before
        if (prev >= 0) {
            {
                std::unique_lock<std::mutex> lk(P->mu);
                P->cv.wait(lk, [&] { return P->err || P->h2d_recorded >= prev; });
                if (P->err) return;
            }
            if (!P->hip_ok(hipEventSynchronize(P->ev_h2d[prev]), "waiting for a staging slot")) return;
        }
        const Piece& pc = B.pieces[j.piece];
        const awq_stream_item& it = P->items[pc.item];
        char* dst = (char*)P->cfg.host_staging + (int64_t)B.slot * P->stride + P->tb + pc.slot_off + j.off;
        const int64_t src = it.offset + pc.row0 * it.K * elem_bytes(it.dtype) + j.off;
        const double t = now_s();
        int64_t done = 0;
        while (done < j.len) {
            const ssize_t got = pread(it.fd, dst + done, (size_t)(j.len - done), (off_t)(src + done));
            if (got < 0 && errno == EINTR) continue;
            if (got <= 0) {
                P->fail(AWQ_EINVAL, "item " + std::to_string(pc.item) + ": read failed at byte " +
                                        std::to_string(src + done) + (got < 0 ? std::string(": ") + strerror(errno)
                                                                              : std::string(": end of file")));
                return;
            }
            done += got;
        }
        std::lock_guard<std::mutex> g(P->mu);
        const double t1 = now_s();
        P->read_busy += t1 - t;
        P->bytes_read += j.len;
        if (!P->tr.empty()) P->tr[j.batch * AWQ_STREAM_TRACE_FIELDS + 1] = t1 - P->t0;
        if (--P->reads_left[j.batch] == 0) P->cv.notify_all();
    }
}

// ---- submitter thread -------------------------------------------------------------------
// outputs of rows [row0, row0 + nrows) of an item
awq_tensor_desc piece_desc(const awq_stream_item& it, const Piece& pc, const void* w, int bits, int64_t gs) {
    const int64_t per = 32 / bits;
    const int64_t wpr = (it.K + per - 1) / per, G = (it.K + gs - 1) / gs, zpr = (G + per - 1) / per;
    awq_tensor_desc d{};
    d.w = w;
    d.rows = pc.nrows;
    d.K = it.K;
    d.qweight = it.qweight ? it.qweight + pc.row0 * wpr : nullptr;
    d.qzeros = it.qzeros ? it.qzeros + pc.row0 * zpr : nullptr;
    d.scales = it.scales ? it.scales + pc.row0 * G : nullptr;
    d.tensor_q = it.tensor_q ? it.tensor_q + pc.row0 * it.K : nullptr;
    d.zeros = it.zeros ? it.zeros + pc.row0 * G : nullptr;
    return d;
}

bool ragged_ok(const awq_tensor_desc& d, int dtype, int64_t gs) {
    return (dtype == AWQ_DTYPE_BF16 || dtype == AWQ_DTYPE_F16 || dtype == AWQ_DTYPE_F32) &&
           awq_ragged_eligible(dtype, d.rows, d.K, gs) && aligned(d.w, 16) && (!d.qweight || aligned(d.qweight, 8)) &&
           (!d.tensor_q || aligned(d.tensor_q, 16)) && (!d.zeros || aligned(d.zeros, 4)) &&
           (!d.qzeros || aligned(d.qzeros, 4)) && (!d.scales || aligned(d.scales, 2));
}

// A batch's launches, planned on the host into the slot's pinned table area (descriptors
// grouped by dtype, then each group's XCD-interleaved tensor table) before the slot's H2D
// carries them to the device together with the input.
struct Group {
    int dtype, first, n;
    int64_t tiles, table_off, table_len;
    int flags;
};
struct BatchPlan {
    std::vector<Group> groups;
    std::vector<std::pair<awq_tensor_desc, int>> rest;   // (descriptor, dtype) of the per-tensor launches
};

bool plan_batch(Pipeline& P, const Batch& B, BatchPlan& bp) {
    const awq_stream_config& c = P.cfg;
    const int64_t gs = c.group_size;
    char* hslot = (char*)c.host_staging + (int64_t)B.slot * P.stride;
    const char* dev_slot = (const char*)c.dev_staging + (int64_t)B.slot * P.stride + P.tb;
    awq_tensor_desc* descs = (awq_tensor_desc*)hslot;   // [AWQ_STREAM_MAX_BATCH_ITEMS], grouped by dtype
    const int64_t tables_at = align_up((int64_t)sizeof(awq_tensor_desc) * AWQ_STREAM_MAX_BATCH_ITEMS, kAlign);
    bp.groups.clear();
    bp.rest.clear();
    int nd = 0;
    int64_t toff = tables_at;
    for (int dt : {AWQ_DTYPE_BF16, AWQ_DTYPE_F16, AWQ_DTYPE_F32, AWQ_DTYPE_F64}) {
        const int first = nd;
        for (const Piece& pc : B.pieces) {
            const awq_stream_item& it = P.items[pc.item];
            if (it.dtype != dt) continue;
            const awq_tensor_desc d = piece_desc(it, pc, dev_slot + pc.slot_off, c.bits, gs);
            if (ragged_ok(d, dt, gs)) descs[nd++] = d;   // (the clip search too: awq_quantize_ragged_search)
            else bp.rest.push_back({d, dt});
        }
        if (nd == first) continue;
        Group g{dt, first, nd - first, 0, 0, 0, 0};
        g.tiles = awq_plan_ragged(descs + first, g.n, c.bits, gs);
        if (g.tiles < 0) {
            P.fail(AWQ_EINVAL, std::string("awq_plan_ragged: ") + awq_last_error());
            return false;
        }
        const int64_t need = awq_plan_block_tensor(descs + first, g.n, g.tiles, nullptr, 0);
        g.table_off = toff;
        g.table_len = need;
        if (toff + need * 4 > P.tb) {
            P.fail(AWQ_EINVAL, "stream tables overflow");
            return false;
        }
        if (need > 0 && awq_plan_block_tensor(descs + first, g.n, g.tiles, (int32_t*)(hslot + toff), need) < 0) {
            P.fail(AWQ_EINVAL, std::string("awq_plan_block_tensor: ") + awq_last_error());
            return false;
        }
        g.flags = awq_ragged_flags(descs + first, g.n, gs);
        toff = align_up(toff + need * 4, 16);
        bp.groups.push_back(g);
    }
    return true;
}

// ph (trace): seconds in the ragged launches and the per-tensor launches
bool launch_batch(Pipeline& P, const Batch& B, const BatchPlan& bp, hipStream_t cs, double (&ph)[2]) {
    const awq_stream_config& c = P.cfg;
    const int64_t gs = c.group_size;
    const char* dslot = (const char*)c.dev_staging + (int64_t)B.slot * P.stride;
    double tp = now_s();
    for (const Group& g : bp.groups) {
        const int32_t* table = g.table_len ? (const int32_t*)(dslot + g.table_off) : nullptr;
        const int rc = c.search_candidates > 1
                           ? awq_quantize_ragged_search((const awq_tensor_desc*)dslot + g.first, g.n, g.tiles, table,
                                                        g.dtype, c.bits, c.symmetric, gs, g.flags, c.search_grid,
                                                        c.search_candidates, cs)
                           : awq_quantize_ragged((const awq_tensor_desc*)dslot + g.first, g.n, g.tiles, table,
                                                 g.dtype, c.bits, c.symmetric, gs, g.flags, cs);
        if (rc) {
            P.fail(rc, std::string("awq_quantize_ragged: ") + awq_last_error());
            return false;
        }
    }
    ph[0] = now_s() - tp;
    tp = now_s();
    for (const auto& r : bp.rest) {
        const awq_tensor_desc& d = r.first;
        const int rc = c.search_candidates > 0
                           ? awq_quantize_search_ex(d.w, r.second, d.rows, d.K, (int32_t)gs, c.bits, c.symmetric, 0,
                                                    c.search_grid, c.search_candidates, d.qweight, d.qzeros, d.scales,
                                                    d.tensor_q, d.zeros, cs)
                           : awq_quantize_groups_ex(d.w, r.second, d.rows, d.K, (int32_t)gs, c.bits, c.symmetric, 0,
                                                    d.qweight, d.qzeros, d.scales, d.tensor_q, d.zeros, cs);
        if (rc) {
            P.fail(rc, std::string(c.search_candidates > 0 ? "awq_quantize_search_ex: " : "awq_quantize_groups_ex: ") +
                           awq_last_error());
            return false;
        }
    }
    ph[1] = now_s() - tp;
    return true;
}

constexpr size_t kWarmBytes = 8 << 20;
constexpr int kMaxDevices = 64;

// HIP's per-process first-use costs, measured in a fresh process (profiles/round4/r4e/
// init.txt): the first stream ~85 ms (the device's first hardware queue), each further one
// ~5 ms, the first H2D of >= 64 KiB ~7 ms, the first launch of a kernel of awq_fast.hip
// ~8.6 ms (its code object is loaded on first use).  warm_main pays them once per device and
// process: three streams (kept for the first pipeline), one 8 MiB H2D, stream-copy launch
// and D2H, then frees its buffers.
struct Warmup {
    std::mutex mu;                      // serialises the start, the join and the pool
    std::thread th;
    bool started = false;
    int err = 0;
    double secs = 0;
    hipStream_t pool[3] = {};           // non-blocking streams made by the warm-up, handed to
    int npool = 0;                      // the device's first pipeline (each further one ~5 ms)
    ~Warmup() {
        if (th.joinable()) th.detach();   // (process exit without awq_runtime_warmup_wait)
    }
};
Warmup g_warm[kMaxDevices];

void warm_main(int device, Warmup* W) {
    const double t = now_s();
    hipStream_t s = nullptr;
    void *h = nullptr, *d = nullptr;
    hipError_t e = hipSetDevice(device);
    for (int k = 0; k < 3 && e == hipSuccess; ++k) {
        e = hipStreamCreateWithFlags(&W->pool[k], hipStreamNonBlocking);
        if (e == hipSuccess) W->npool = k + 1;
    }
    if (e == hipSuccess) s = W->pool[0];
    if (e == hipSuccess) e = hipHostMalloc(&h, kWarmBytes, 0);
    if (e == hipSuccess) e = hipMalloc(&d, kWarmBytes);
    if (e == hipSuccess) e = hipMemcpyAsync(d, h, kWarmBytes, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = awq::launch_stream_copy(d, (char*)d + kWarmBytes / 2, kWarmBytes / 2, s);
    if (e == hipSuccess) e = hipMemcpyAsync(h, d, kWarmBytes, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) {                // (no pool after a failure: the pipeline makes its own)
        for (int k = 0; k < W->npool; ++k) (void)hipStreamDestroy(W->pool[k]);
        W->npool = 0;
    }
    if (h) (void)hipHostFree(h);
    if (d) (void)hipFree(d);
    W->err = e == hipSuccess ? 0 : AWQ_EHIP;
    W->secs = now_s() - t;
}

// The pipeline's device side: the device's first-use warm-up (joined if a caller started it
// early with awq_runtime_warmup, else run here), then the streams the caller left NULL
// (non-blocking) — all on the submitter thread, while the readers fill the first slots.
bool prepare_device(Pipeline* P) {
    struct {
        hipStream_t* s;
        bool own;
    } st[3] = {{&P->st_h2d, P->own_h2d}, {&P->st_cs, P->own_cs}, {&P->st_d2h, P->own_d2h}};
    if (P->device >= 0 && P->device < kMaxDevices) {
        Warmup& W = g_warm[P->device];
        std::lock_guard<std::mutex> g(W.mu);
        if (!W.started) {
            W.started = true;
            warm_main(P->device, &W);
        } else if (W.th.joinable()) {
            W.th.join();
        }
        (void)hipSetDevice(P->device);
        for (auto& e : st)                // the warm-up's streams first (already created)
            if (e.own && W.npool > 0) *e.s = W.pool[--W.npool];
    }
    for (auto& e : st)
        if (e.own && !*e.s && !P->hip_ok(hipStreamCreateWithFlags(e.s, hipStreamNonBlocking), "hipStreamCreate"))
            return false;
    if (!P->tr.empty()) {
        if (!P->hip_ok(hipEventCreate(&P->ev_start), "trace event") ||
            !P->hip_ok(hipEventRecord(P->ev_start, P->st_h2d), "trace event"))
            return false;
        P->ev_start_host = now_s() - P->t0;
    }
    return true;
}

void submitter_main(Pipeline* P) {
    (void)hipSetDevice(P->device);
    const awq_stream_config& c = P->cfg;
    const double tp = now_s();
    if (!prepare_device(P)) return;
    P->prepare = now_s() - tp;
    hipStream_t h2d = P->st_h2d, cs = P->st_cs, d2h = P->st_d2h;
    const int64_t nb = (int64_t)P->batches.size();
    BatchPlan bp;
    for (int64_t b = 0; b < nb; ++b) {
        const Batch& B = P->batches[b];
        double t = now_s();
        {
            std::unique_lock<std::mutex> lk(P->mu);
            P->cv.wait(lk, [&] { return P->err || P->abort || P->reads_left[b] == 0; });
            if (P->err) return;
            if (P->abort) {
                lk.unlock();
                P->fail(AWQ_EINVAL, "stream cancelled (awq_stream_end before its last batch)");
                return;
            }
        }
        P->wait_read += now_s() - t;
        double t_slot = 0;
        if (b >= c.nslots) {   // the slot's previous batch: its kernels read the device slot and its tables
            t = now_s();
            if (!P->hip_ok(hipEventSynchronize(P->ev_kern[b - c.nslots]), "waiting for a slot's kernels")) return;
            t_slot = now_s() - t;
            P->wait_slot += t_slot;
        }
        // plan the launches into the slot's table area (the slot's previous kernels are done:
        // its device tables are free, and its H2D is done: so are the host ones)
        double t_plan = now_s();
        if (!plan_batch(*P, B, bp)) return;
        t_plan = now_s() - t_plan;
        const double t_h2d = now_s();
        if (!P->hip_ok(hipMemcpyAsync((char*)c.dev_staging + (int64_t)B.slot * P->stride,
                                      (const char*)c.host_staging + (int64_t)B.slot * P->stride,
                                      (size_t)(P->tb + B.bytes), hipMemcpyHostToDevice, h2d),
                       "H2D"))
            return;
        if (!P->hip_ok(hipEventRecord(P->ev_h2d[b], h2d), "event")) return;
        if (!P->tr.empty()) {
            P->tr[b * AWQ_STREAM_TRACE_FIELDS + 2] = now_s() - P->t0;
            P->tr[b * AWQ_STREAM_TRACE_FIELDS + 8] = now_s() - t_h2d;
            P->tr[b * AWQ_STREAM_TRACE_FIELDS + 10] = t_plan;
            P->tr[b * AWQ_STREAM_TRACE_FIELDS + 11] = t_slot;
        }
        {
            std::lock_guard<std::mutex> g(P->mu);
            P->h2d_recorded = b;
        }
        P->cv.notify_all();
        if (!P->hip_ok(hipStreamWaitEvent(cs, P->ev_h2d[b], 0), "stream wait")) return;
        // device output ring: the ranges this batch's kernels overwrite have been copied back
        if (B.dev_wait >= 0 && !P->hip_ok(hipStreamWaitEvent(cs, P->ev_done[B.dev_wait], 0), "stream wait")) return;
        double ph[2] = {0, 0};
        if (!launch_batch(*P, B, bp, cs, ph)) return;
        if (!P->tr.empty())
            for (int k = 0; k < 2; ++k) P->tr[b * AWQ_STREAM_TRACE_FIELDS + 12 + k] = ph[k];
        if (!P->hip_ok(hipEventRecord(P->ev_kern[b], cs), "event")) return;
        if (!P->tr.empty()) P->tr[b * AWQ_STREAM_TRACE_FIELDS + 3] = now_s() - P->t0;
        if (!P->hip_ok(hipStreamWaitEvent(d2h, P->ev_kern[b], 0), "stream wait")) return;
        // host output ring: the caller has released the ranges this batch's D2H overwrites
        if (B.host_gate > 0) {
            const double tw = now_s();
            std::unique_lock<std::mutex> lk(P->mu);
            P->cv.wait(lk, [&] { return P->err || P->abort || P->released >= B.host_gate; });
            if (P->err) return;
            if (P->abort) {
                lk.unlock();
                P->fail(AWQ_EINVAL, "stream cancelled (awq_stream_end before its last batch)");
                return;
            }
            P->wait_release += now_s() - tw;
        }
        // outputs of the items this batch completes (two ranges per item), adjacent ranges as
        // one copy
        struct Run {
            char *hs = nullptr, *ds = nullptr;
            int64_t len = 0;
        } run[2];
        double t_d2h = 0;
        auto flush = [&](Run& r) {
            const double tc = now_s();
            if (r.len > 0 && !P->hip_ok(hipMemcpyAsync(r.hs, r.ds, (size_t)r.len, hipMemcpyDeviceToHost, d2h), "D2H"))
                return false;
            t_d2h += now_s() - tc;
            r.len = 0;
            return true;
        };
        for (int i = B.item_begin; i < B.item_end; ++i) {
            const awq_stream_item& it = P->items[i];
            const void* h[2] = {it.host_out, it.host_out2};
            const void* dv[2] = {it.dev_out, it.dev_out2};
            const int64_t nb[2] = {it.out_bytes, it.out_bytes2};
            for (int k = 0; k < 2; ++k) {
                if (!h[k] || !dv[k] || nb[k] <= 0) continue;
                Run& r = run[k];
                if (r.len > 0 && r.hs + r.len == (const char*)h[k] && r.ds + r.len == (const char*)dv[k]) {
                    r.len += nb[k];
                    continue;
                }
                if (!flush(r)) return;
                r.hs = (char*)h[k];
                r.ds = (char*)dv[k];
                r.len = nb[k];
            }
        }
        if (!flush(run[0]) || !flush(run[1])) return;
        if (!P->hip_ok(hipEventRecord(P->ev_done[b], d2h), "event")) return;
        if (!P->tr.empty()) {
            P->tr[b * AWQ_STREAM_TRACE_FIELDS + 4] = now_s() - P->t0;
            P->tr[b * AWQ_STREAM_TRACE_FIELDS + 9] = t_d2h;
        }
        {
            std::lock_guard<std::mutex> g(P->mu);
            P->done_recorded = b;
        }
        P->cv.notify_all();
    }
}

}  // namespace

namespace awq {
int set_error(int code, const char* msg);   // awq_capi.hip
}

extern "C" {

int64_t awq_stream_table_bytes(int64_t slot_bytes) {
    const int64_t descs = align_up((int64_t)sizeof(awq_tensor_desc) * AWQ_STREAM_MAX_BATCH_ITEMS, kAlign);
    // tensor tables: one 64-B entry per AWQ_BLOCK_TILES tiles of >= 4 KiB of input, per dtype group
    const int64_t tables = 64 * (slot_bytes / 4096 / AWQ_BLOCK_TILES + 4 * 16) + 4 * 16;
    return align_up(descs + tables, 4096);
}

int awq_stream_start(const awq_stream_item* items, int n, const awq_stream_config* cfg, void** handle) {
    if (!handle || !cfg || n < 0 || (n > 0 && !items)) return awq::set_error(AWQ_EINVAL, "null argument");
    *handle = nullptr;
    const awq_stream_config& c = *cfg;
    if (c.bits != 4 && c.bits != 8) return awq::set_error(AWQ_EINVAL, "Unsupported bit width. Supported: 4, 8.");
    if (c.group_size <= 0) return awq::set_error(AWQ_EINVAL, "Group size must be a positive integer");
    if (c.nslots < 2 || c.readers < 1 || c.slot_bytes <= 0 || c.slot_bytes % 4096 || !c.host_staging ||
        !c.dev_staging)
        return awq::set_error(AWQ_EINVAL, "bad stream configuration (nslots >= 2, readers >= 1, slot_bytes a "
                                          "multiple of 4096, staging buffers)");
    if (c.search_candidates < 0 || (c.search_candidates > 0 && (c.search_grid < 1 || c.search_candidates > c.search_grid)))
        return awq::set_error(AWQ_EINVAL, "bad search configuration (1 <= search_candidates <= search_grid)");
    for (int i = 0; i < n; ++i) {
        const awq_stream_item& it = items[i];
        if (it.dtype < AWQ_DTYPE_BF16 || it.dtype > AWQ_DTYPE_F64 || it.rows < 0 || it.K < 0 || it.fd < 0 ||
            it.offset < 0)
            return awq::set_error(AWQ_EINVAL, ("item " + std::to_string(i) + ": bad dtype, shape, fd or offset").c_str());
        if (!it.qweight && !it.qzeros && !it.scales && !it.tensor_q && !it.zeros)
            return awq::set_error(AWQ_EINVAL, "an item requests no output");
    }
    Pipeline* P = new Pipeline();
    P->items.assign(items, items + n);
    P->cfg = c;
    P->tb = awq_stream_table_bytes(c.slot_bytes);
    P->stride = P->tb + c.slot_bytes;
    (void)hipGetDevice(&P->device);
    std::string why;
    if (int rc = plan(*P, why)) {
        delete P;
        return awq::set_error(rc, why.c_str());
    }
    const size_t nb = P->batches.size();
    P->ev_h2d.resize(nb);
    P->ev_kern.resize(nb);
    P->ev_done.resize(nb);
    const bool trace = c.trace != nullptr && c.trace_batches > 0;
    for (size_t b = 0; b < nb; ++b)
        for (hipEvent_t* e : {&P->ev_h2d[b], &P->ev_kern[b], &P->ev_done[b]})
            if (hipEventCreateWithFlags(e, trace ? hipEventDefault : hipEventDisableTiming) != hipSuccess) {
                delete P;   // (events created so far are reclaimed with the context)
                return awq::set_error(AWQ_EHIP, "hipEventCreate failed");
            }
    if (trace) P->tr.assign(nb * AWQ_STREAM_TRACE_FIELDS, -1.0);
    P->st_cs = (hipStream_t)c.compute_stream;
    P->st_h2d = (hipStream_t)c.h2d_stream;
    P->st_d2h = (hipStream_t)c.d2h_stream;
    P->own_cs = !P->st_cs;
    P->own_h2d = !P->st_h2d;
    P->own_d2h = !P->st_d2h;
    P->t0 = now_s();
    const int nr = std::max(1, std::min(c.readers, (int)std::max<size_t>(1, P->jobs.size())));
    for (int r = 0; r < nr; ++r) P->readers.emplace_back(reader_main, P);
    P->submitter = std::thread(submitter_main, P);
    *handle = P;
    return AWQ_OK;
}

int awq_runtime_warmup(int device) {
    if (device < 0 || device >= kMaxDevices) return awq::set_error(AWQ_EINVAL, "bad device index");
    Warmup& W = g_warm[device];
    std::lock_guard<std::mutex> g(W.mu);
    if (!W.started) {
        W.started = true;
        W.th = std::thread(warm_main, device, &W);
    }
    return AWQ_OK;
}

int awq_runtime_warmup_wait(int device, double* seconds) {
    if (device < 0 || device >= kMaxDevices) return awq::set_error(AWQ_EINVAL, "bad device index");
    Warmup& W = g_warm[device];
    std::lock_guard<std::mutex> g(W.mu);
    if (W.th.joinable()) W.th.join();
    if (seconds) *seconds = W.secs;
    return W.err ? awq::set_error(W.err, "device warm-up failed") : AWQ_OK;
}

int64_t awq_stream_plan(const awq_stream_item* items, int n, const awq_stream_config* cfg, int32_t* first_batch,
                        int32_t* last_batch) {
    if (!cfg || n < 0 || (n > 0 && !items)) return -awq::set_error(AWQ_EINVAL, "null argument");
    if (cfg->nslots < 1 || cfg->slot_bytes <= 0) return -awq::set_error(AWQ_EINVAL, "bad stream configuration");
    Pipeline P;
    P.items.assign(items, items + n);
    P.cfg = *cfg;
    std::string why;
    if (int rc = plan(P, why)) return -awq::set_error(rc, why.c_str());
    for (int i = 0; i < n; ++i) {
        if (first_batch) first_batch[i] = P.first_batch[i];
        if (last_batch) last_batch[i] = P.last_batch[i];
    }
    return (int64_t)P.batches.size();
}

int awq_stream_release(void* handle, int32_t items) {
    Pipeline* P = (Pipeline*)handle;
    if (!P) return awq::set_error(AWQ_EINVAL, "null handle");
    {
        std::lock_guard<std::mutex> g(P->mu);
        P->released = std::max(P->released, items);
    }
    P->cv.notify_all();
    return AWQ_OK;
}

int64_t awq_stream_batches(void* handle) {
    return handle ? (int64_t)((Pipeline*)handle)->batches.size() : -1;
}

int awq_stream_wait(void* handle, int64_t batch, int32_t* first_item, int32_t* end_item) {
    Pipeline* P = (Pipeline*)handle;
    if (!P || batch < 0 || batch >= (int64_t)P->batches.size()) return awq::set_error(AWQ_EINVAL, "bad batch");
    {
        std::unique_lock<std::mutex> lk(P->mu);
        P->cv.wait(lk, [&] { return P->err || P->done_recorded >= batch; });
        if (P->err) return awq::set_error(P->err, P->err_msg.c_str());
    }
    const hipError_t e = hipEventSynchronize(P->ev_done[batch]);
    if (e != hipSuccess) return awq::set_error(AWQ_EHIP, hipGetErrorString(e));
    if (first_item) *first_item = P->batches[batch].item_begin;
    if (end_item) *end_item = P->batches[batch].item_end;
    return AWQ_OK;
}

int awq_stream_end(void* handle, awq_stream_stats* stats) {
    Pipeline* P = (Pipeline*)handle;
    if (!P) return awq::set_error(AWQ_EINVAL, "null handle");
    {   // a caller that stopped early may still read its host ranges: copy nothing more into them
        std::lock_guard<std::mutex> g(P->mu);
        P->abort = true;
    }
    P->cv.notify_all();
    if (P->submitter.joinable()) P->submitter.join();
    {   // a failed submitter leaves readers waiting for slots: release them
        std::lock_guard<std::mutex> g(P->mu);
        if (P->done_recorded + 1 < (int64_t)P->batches.size() && !P->err) {
            P->err = AWQ_EHIP;
            P->err_msg = "stream pipeline stopped early";
        }
        P->cv.notify_all();
    }
    for (auto& t : P->readers) t.join();
    int rc = P->err;
    std::string msg = P->err_msg;
    if (!rc && !P->batches.empty()) {
        const hipError_t e = hipEventSynchronize(P->ev_done.back());
        if (e != hipSuccess) {
            rc = AWQ_EHIP;
            msg = hipGetErrorString(e);
        }
    }
    if (stats) {
        stats->batches = (int64_t)P->batches.size();
        int64_t pieces = 0;
        for (const Batch& b : P->batches) pieces += (int64_t)b.pieces.size();
        stats->pieces = pieces;
        stats->bytes_read = P->bytes_read;
        stats->wall_s = now_s() - P->t0;
        stats->read_busy_s = P->read_busy;
        stats->wait_read_s = P->wait_read;
        stats->wait_slot_s = P->wait_slot;
        stats->wait_release_s = P->wait_release;
        stats->prepare_s = P->prepare;
    }
    // nothing of the pipeline may still run once the caller's buffers are released
    const struct {
        hipStream_t s;
        bool own;
    } streams[3] = {{P->st_h2d, P->own_h2d}, {P->st_cs, P->own_cs}, {P->st_d2h, P->own_d2h}};
    for (const auto& e : streams)
        if (e.s || !e.own) (void)hipStreamSynchronize(e.s);   // (an own stream not created: nothing ran)
    if (P->ev_start) {
        const size_t nt = std::min(P->batches.size(), (size_t)P->cfg.trace_batches);
        for (size_t b = 0; b < nt; ++b) {
            double* o = P->cfg.trace + b * AWQ_STREAM_TRACE_FIELDS;
            for (int k = 0; k < 5; ++k) o[k] = P->tr[b * AWQ_STREAM_TRACE_FIELDS + k];
            for (int k = 8; k < AWQ_STREAM_TRACE_FIELDS; ++k) o[k] = P->tr[b * AWQ_STREAM_TRACE_FIELDS + k];
            const hipEvent_t ev[3] = {P->ev_h2d[b], P->ev_kern[b], P->ev_done[b]};
            for (int k = 0; k < 3; ++k) {
                float ms = -1.0f;
                o[5 + k] = (!rc && hipEventElapsedTime(&ms, P->ev_start, ev[k]) == hipSuccess)
                               ? P->ev_start_host + ms * 1e-3 : -1.0;
            }
        }
        (void)hipEventDestroy(P->ev_start);
    }
    for (size_t b = 0; b < P->batches.size(); ++b) {
        (void)hipEventDestroy(P->ev_h2d[b]);
        (void)hipEventDestroy(P->ev_kern[b]);
        (void)hipEventDestroy(P->ev_done[b]);
    }
    for (const auto& e : streams)
        if (e.own && e.s) (void)hipStreamDestroy(e.s);
    delete P;
    if (rc) return awq::set_error(rc, msg.c_str());
    return AWQ_OK;
}

}  // extern "C"
