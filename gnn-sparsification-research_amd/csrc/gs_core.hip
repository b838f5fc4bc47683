// gs_core.hip -- context lifecycle, errors, profiling, copies, device-wide
// primitives (rocPRIM radix sort / scan) for libgsparse.
#include <cstdarg>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "gs_internal.hpp"

namespace gs {

static thread_local char g_err[1024] = "";

void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

hipEvent_t prof_begin(gs_ctx *c) {
    if (!c->profiling) return nullptr;
    hipEvent_t e;
    GS_HIP(hipEventCreate(&e));
    GS_HIP(hipEventRecord(e, c->stream));
    return e;
}

void prof_end(gs_ctx *c, hipEvent_t start, const char *name, double bytes) {
    if (!c->profiling || !start) return;
    hipEvent_t e;
    GS_HIP(hipEventCreate(&e));
    GS_HIP(hipEventRecord(e, c->stream));
    c->pending.push_back(ProfPending{name, start, e, bytes});
    if (c->pending.size() >= (size_t)kProfPendingMax) prof_flush(c);
}

void prof_note(gs_ctx *c, const char *name) {
    if (!c->profiling) return;
    auto it = c->prof.find(name);
    if (it == c->prof.end()) {
        c->prof_order.push_back(name);
        it = c->prof.emplace(name, ProfEntry{}).first;
    }
    it->second.launches += 1;
}

void prof_flush(gs_ctx *c) {
    split_abort_poll(c, true);
    if (c->pending.empty()) return;
    GS_HIP(hipStreamSynchronize(c->stream));
    bool slots = false;
    for (auto &p : c->pending) slots = slots || p.its_slot >= 0;
    if (slots) {
        std::vector<int64_t> its(c->pending.size(), 0);
        GS_HIP(hipMemcpy(its.data(), c->buf("prof_its").as<int64_t>(), sizeof(int64_t) * its.size(),
                         hipMemcpyDeviceToHost));
        for (auto &p : c->pending)
            if (p.its_slot >= 0) p.bytes += p.its_bytes * (double)its[(size_t)p.its_slot];
    }
    for (auto &p : c->pending) {
        float ms = 0.f;
        GS_HIP(hipEventElapsedTime(&ms, p.start, p.stop));
        auto it = c->prof.find(p.name);
        if (it == c->prof.end()) {
            c->prof_order.push_back(p.name);
            it = c->prof.emplace(p.name, ProfEntry{}).first;
        }
        it->second.launches += 1;
        it->second.ms += ms;
        it->second.bytes += p.bytes;
        (void)hipEventDestroy(p.start);
        (void)hipEventDestroy(p.stop);
    }
    c->pending.clear();
}

void sync_if_needed(gs_ctx *c) {
    if (!c->async_) GS_HIP(hipStreamSynchronize(c->stream));
}

const void *to_device(gs_ctx *c, DevBuf &buf, const void *p, size_t bytes, int loc) {
    if (loc == GS_DEVICE || bytes == 0) return p;
    void *d = buf.ensure(bytes);
    GS_HIP(hipMemcpyAsync(d, p, bytes, hipMemcpyHostToDevice, c->stream));
    return d;
}

void *out_device(gs_ctx *c, DevBuf &buf, void *p, size_t bytes, int loc) {
    if (loc == GS_DEVICE) return p;
    return buf.ensure(bytes);
}

void finish_out(gs_ctx *c, void *host, const void *dev, size_t bytes, int loc) {
    if (loc == GS_DEVICE) {
        sync_if_needed(c);
        return;
    }
    if (bytes) GS_HIP(hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, c->stream));
    GS_HIP(hipStreamSynchronize(c->stream));
}

void exclusive_scan_i64(gs_ctx *c, const int64_t *in, int64_t *out, int64_t n) {
    if (n <= 0) return;
    size_t tmp = 0;
    GS_HIP(rocprim::exclusive_scan(nullptr, tmp, in, out, (int64_t)0, (size_t)n,
                                   rocprim::plus<int64_t>(), c->stream));
    void *t = c->scratch[5].ensure(tmp + 16);
    GS_HIP(rocprim::exclusive_scan(t, tmp, in, out, (int64_t)0, (size_t)n,
                                   rocprim::plus<int64_t>(), c->stream));
}

void sort_keys_u64(gs_ctx *c, uint64_t *keys, int64_t n, int end_bit) {
    if (n <= 1) return;
    DevBuf &alt = c->scratch[4];
    uint64_t *k2 = (uint64_t *)alt.ensure(sizeof(uint64_t) * n);
    rocprim::double_buffer<uint64_t> db(keys, k2);
    size_t tmp = 0;
    GS_HIP(rocprim::radix_sort_keys(nullptr, tmp, db, (size_t)n, 0, end_bit, c->stream));
    void *t = c->scratch[5].ensure(tmp + 16);
    GS_HIP(rocprim::radix_sort_keys(t, tmp, db, (size_t)n, 0, end_bit, c->stream));
    if (db.current() != keys)
        GS_HIP(hipMemcpyAsync(keys, db.current(), sizeof(uint64_t) * n, hipMemcpyDeviceToDevice,
                              c->stream));
}

void sort_pairs_u64_i64(gs_ctx *c, uint64_t *keys, int64_t *vals, int64_t n, int end_bit) {
    if (n <= 1) return;
    DevBuf &alt = c->scratch[4];
    DevBuf &altv = c->scratch[3];
    uint64_t *k2 = (uint64_t *)alt.ensure(sizeof(uint64_t) * n);
    int64_t *v2 = (int64_t *)altv.ensure(sizeof(int64_t) * n);
    rocprim::double_buffer<uint64_t> dk(keys, k2);
    rocprim::double_buffer<int64_t> dv(vals, v2);
    size_t tmp = 0;
    GS_HIP(rocprim::radix_sort_pairs(nullptr, tmp, dk, dv, (size_t)n, 0, end_bit, c->stream));
    void *t = c->scratch[5].ensure(tmp + 16);
    GS_HIP(rocprim::radix_sort_pairs(t, tmp, dk, dv, (size_t)n, 0, end_bit, c->stream));
    if (dk.current() != keys) {
        GS_HIP(hipMemcpyAsync(keys, dk.current(), sizeof(uint64_t) * n, hipMemcpyDeviceToDevice,
                              c->stream));
        GS_HIP(hipMemcpyAsync(vals, dv.current(), sizeof(int64_t) * n, hipMemcpyDeviceToDevice,
                              c->stream));
    }
}

}  // namespace gs

using namespace gs;

namespace gs {
void jsel_forget(gs_ctx *c);  // gs_jsel.hip: drop the select state kept for this context
}

extern "C" {

int gs_api_version(void) { return GS_API_VERSION; }

const char *gs_last_error(void) { return g_err; }

int gs_device_count(int *count) {
    return guard([&] {
        int n = 0;
        GS_HIP(hipGetDeviceCount(&n));
        *count = n;
    });
}

int gs_create(int device, gs_ctx **out) {
    return guard([&] {
        GS_CHECK(out, GS_EINVAL, "gs_create: out is NULL");
        int n = 0;
        GS_HIP(hipGetDeviceCount(&n));
        GS_CHECK(device >= 0 && device < n, GS_EINVAL, "gs_create: device %d of %d", device, n);
        GS_HIP(hipSetDevice(device));
        hipDeviceProp_t prop;
        GS_HIP(hipGetDeviceProperties(&prop, device));
        GS_CHECK(strncmp(prop.gcnArchName, "gfx950", 6) == 0, GS_EUNSUPPORTED,
                 "libgsparse is built for gfx950 (MI355X); device %d is %s", device,
                 prop.gcnArchName);
        gs_ctx *c = new gs_ctx();
        c->device = device;
        GS_HIP(hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking));
        c->stream = c->own_stream;
        *out = c;
    });
}

void gs_destroy(gs_ctx *c) {
    if (!c) return;
    gs::jsel_forget(c);
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    for (auto &p : c->pending) {
        (void)hipEventDestroy(p.start);
        (void)hipEventDestroy(p.stop);
    }
    DevBuf *gb[] = {&c->g.indptr, &c->g.indices, &c->g.data, &c->g.rows, &c->g.tptr,
                    &c->g.tidx,   &c->g.tpos};
    for (auto *b : gb) b->release();
    DevBuf *eb[] = {&c->er.edge_id, &c->er.bptr, &c->er.bcol, &c->er.bsgn, &c->er.bcur,
                    &c->er.lp,      &c->er.li,   &c->er.lv,   &c->er.X,    &c->er.Rr,
                    &c->er.P0,      &c->er.P1,   &c->er.Q,    &c->er.colstate,
                    &c->er.acc,     &c->er.iters, &c->er.rawbuf};
    for (auto *b : eb) b->release();
    for (auto &b : c->scratch) b.release();
    for (auto &kv : c->named) kv.second.release();
    c->outbuf.release();
    c->inbuf.release();
    c->inbuf2.release();
    for (auto &a : c->aux)
        if (a) (void)hipStreamDestroy(a);
    for (auto &e : c->aux_ev)
        if (e) (void)hipEventDestroy(e);
    if (c->order_ev) (void)hipEventDestroy(c->order_ev);
    if (c->split_abort_ev) (void)hipEventDestroy(c->split_abort_ev);
    if (c->split_abort_host) (void)hipHostFree(c->split_abort_host);
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    delete c;
}

int gs_set_stream(gs_ctx *c, void *s) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        GS_HIP(hipSetDevice(c->device));
        c->stream = s ? (hipStream_t)s : c->own_stream;
    });
}

// Cross-stream ordering with a caller's stream (e.g. torch's current stream):
// an event recorded on the producer, waited on by the consumer -- no host sync.
static void order_streams(gs_ctx *c, hipStream_t producer, hipStream_t consumer) {
    GS_HIP(hipSetDevice(c->device));
    if (producer == consumer) return;
    if (!c->order_ev) GS_HIP(hipEventCreateWithFlags(&c->order_ev, hipEventDisableTiming));
    GS_HIP(hipEventRecord(c->order_ev, producer));
    GS_HIP(hipStreamWaitEvent(consumer, c->order_ev, 0));
}

int gs_stream_wait(gs_ctx *c, void *s) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        order_streams(c, (hipStream_t)s, c->stream);
    });
}

int gs_stream_signal(gs_ctx *c, void *s) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        order_streams(c, c->stream, (hipStream_t)s);
    });
}

int gs_synchronize(gs_ctx *c) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        GS_HIP(hipStreamSynchronize(c->stream));
        split_abort_poll(c, true);
    });
}

int gs_set_async(gs_ctx *c, int a) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        c->async_ = a != 0;
    });
}

int gs_profile_enable(gs_ctx *c, int on) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        c->profiling = on != 0;
    });
}

int gs_profile_reset(gs_ctx *c) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        prof_flush(c);
        c->prof.clear();
        c->prof_order.clear();
    });
}

int gs_profile_get(gs_ctx *c, int i, char *name, int name_len, int64_t *launches, double *ms,
                   double *bytes) {
    int rc = guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        prof_flush(c);
    });
    if (rc) return rc;
    if (i < 0 || i >= (int)c->prof_order.size()) return -1;
    const std::string &nm = c->prof_order[i];
    const ProfEntry &e = c->prof[nm];
    if (name && name_len > 0) {
        strncpy(name, nm.c_str(), name_len - 1);
        name[name_len - 1] = 0;
    }
    if (launches) *launches = e.launches;
    if (ms) *ms = e.ms;
    if (bytes) *bytes = e.bytes;
    return GS_OK;
}

}  // extern "C"
