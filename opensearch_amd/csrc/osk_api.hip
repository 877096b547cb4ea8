// osk_api.hip — the C-ABI of libosknn.so (declared in include/osknn.h): segments, views, the
// single-device search paths and the coordinator merge.  The object model (osk_seg, osk_view) is in
// osk_objects.h; the multi-GPU exchange (osk_comm, RCCL) in osk_comm.hip.
// Every entry point catches all C++ exceptions and returns an error code (see osknn.h).
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cerrno>
#include <cstring>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <vector>

#include "osk_objects.h"

using namespace osk;

namespace {
std::mutex g_dev_mu;
std::vector<hipStream_t> g_streams;
int g_ndev = -1;
// Per-call device time of this thread's last synchronous host search (osk_last_call_device_ns):
// nanoseconds between the call's first and last device operation on its stream, and how many host
// requests shared that launch chain (opportunistic batching).  −1 / 0: timing off or no call yet.
thread_local int64_t t_call_ns = -1;
thread_local int32_t t_call_shared = 0;

// Call timing of a host search (tune "call_timing"): events bracket the call's work on its stream.
struct CallTimer {
    osk_view* v = nullptr;
    hipStream_t st = nullptr;
    int32_t begin(osk_view* view, hipStream_t stream) {
        t_call_ns = -1;
        t_call_shared = 0;
        if (!g_tuning.call_timing) return OSK_OK;
        for (hipEvent_t& e : view->ev_call)
            if (!e) OSK_HIP(hipEventCreate(&e));
        v = view;
        st = stream;
        OSK_HIP(hipEventRecord(v->ev_call[0], st));
        return OSK_OK;
    }
    int32_t end() {   // before the call's final stream synchronisation
        if (v) OSK_HIP(hipEventRecord(v->ev_call[1], st));
        return OSK_OK;
    }
    int32_t publish() {   // after it
        if (!v) return OSK_OK;
        float ms = 0.f;
        OSK_HIP(hipEventElapsedTime(&ms, v->ev_call[0], v->ev_call[1]));
        t_call_ns = (int64_t)((double)ms * 1e6);
        t_call_shared = 1;
        return OSK_OK;
    }
};
}  // namespace

namespace osk {

// ------------------------------------------------------------------------------------------------
// devices and streams
// ------------------------------------------------------------------------------------------------

int device_count_cached() {
    std::lock_guard<std::mutex> lk(g_dev_mu);
    if (g_ndev < 0) {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
        g_ndev = n;
        g_streams.assign(n, nullptr);
    }
    return g_ndev;
}

int32_t check_device(int device) {
    const int n = device_count_cached();
    if (n <= 0) {
        set_error("no HIP device visible (libosknn has no CPU fallback)");
        return OSK_ERR_NO_DEVICE;
    }
    if (device < 0 || device >= n) {
        set_error("device index out of range");
        return OSK_ERR_INVALID;
    }
    static std::atomic<int> arch_ok[64];   // per device: 0 unknown, 1 gfx950, 2 another arch
    if (device >= 64 || arch_ok[device].load() == 0) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, device) != hipSuccess) {
            set_error("hipGetDeviceProperties failed");
            return OSK_ERR_DEVICE;
        }
        const bool ok = std::strncmp(prop.gcnArchName, "gfx950", 6) == 0;
        if (device < 64) arch_ok[device].store(ok ? 1 : 2);
        if (!ok) {
            set_error(std::string("device is ") + prop.gcnArchName + ", libosknn is built for gfx950");
            return OSK_ERR_NO_DEVICE;
        }
    } else if (arch_ok[device].load() == 2) {
        set_error("device is not gfx950; libosknn is built for gfx950");
        return OSK_ERR_NO_DEVICE;
    }
    if (hipSetDevice(device) != hipSuccess) {
        set_error("hipSetDevice failed");
        return OSK_ERR_DEVICE;
    }
    return OSK_OK;
}

hipStream_t device_stream(int device) {
    std::lock_guard<std::mutex> lk(g_dev_mu);
    if (!g_streams[device]) {
        hipStream_t s;
        if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return nullptr;
        g_streams[device] = s;
    }
    return g_streams[device];
}


// The device view of a view's segments (pointers re-read: staging may add row norms later).
std::vector<SegDev> seg_devs(const osk_view* v) {
    std::vector<SegDev> sd(v->segs.size());
    for (size_t i = 0; i < v->segs.size(); ++i) {
        const osk_seg* s = v->segs[i];
        sd[i] = SegDev{s->d_rows, s->d_xnorm_f, s->d_xnorm_i, s->d_ord_to_doc, s->n_rows,
                       v->seg_doc_base[i], v->seg_shard[i]};
    }
    return sd;
}

}  // namespace osk

namespace {
void sq6_forget_segment(const osk_seg* sg);   // (below, with the 6-bit tier's in-flight records)
}

osk_seg::~osk_seg() {
    if (self_view) delete self_view;   // holds no reference on this segment
    if (d_rows) (void)hipFree(d_rows);
    if (d_xnorm_f) (void)hipFree(d_xnorm_f);
    if (d_xnorm_i) (void)hipFree(d_xnorm_i);
    if (d_ord_to_doc) (void)hipFree(d_ord_to_doc);
    if (d_split) (void)hipFree(d_split);
    if (d_maxnorm2) (void)hipFree(d_maxnorm2);
    if (d_xsqrt) (void)hipFree(d_xsqrt);
    if (d_q8) (void)hipFree(d_q8);
    if (d_q8aux) (void)hipFree(d_q8aux);
    if (d_q8t) (void)hipFree(d_q8t);
    if (d_q8auxt) (void)hipFree(d_q8auxt);
    if (d_q8w) (void)hipFree(d_q8w);
    if (d_q6 || d_q6aux) {   // stream-ordered pool allocations (ensure_sq8_seg); the hipFree calls above
        int cur = -1;         // synchronised the device, so nothing reads them any more
        (void)hipGetDevice(&cur);
        (void)hipSetDevice(device);
        if (d_q6) (void)hipFreeAsync(d_q6, nullptr);
        if (d_q6aux) (void)hipFreeAsync(d_q6aux, nullptr);
        (void)hipStreamSynchronize(nullptr);
        if (cur >= 0) (void)hipSetDevice(cur);
    }
    sq6_forget_segment(this);   // (a later segment at this address must not wait on this one's launches)
}

int64_t osk_seg::hbm_bytes() const {
    const int64_t n = std::max<int64_t>(1, n_rows);
    int64_t b = n * units * 16;
    if (d_xnorm_f) b += n * 4;
    if (d_xnorm_i) b += n * 4;
    if (d_ord_to_doc) b += n * 4;
    if (d_split) b += std::max<int64_t>(1, (n_rows + 127) / 128) * 8 * split_KS * 2 * 1024 + n * 4 + 4;
    if (d_q8) b += n * units8 * 16 + n * 16;
    if (d_q8t) b += std::max<int64_t>(1, (n_rows + 15) / 16) * sq8_mfma_ks(units8) * 1024;
    if (d_q8auxt) b += std::max<int64_t>(1, (n_rows + 15) / 16) * kAuxGroupF4 * 16;
    if (d_q8w) b += std::max<int64_t>(1, (n_rows + 15) / 16) * sq8_wide_ks(units8) * 1024;
    if (d_q6) b += sq6_bytes(n_rows, dim);
    return b;
}

osk_view::~osk_view() {
    for (osk_view* r : replicas) delete r;   // (no lease is live: the caller's release contract)
    for (hipStream_t st : lease_streams)
        if (st) (void)hipStreamDestroy(st);
    if (xs_event) (void)hipEventDestroy(xs_event);
    if (ev_probe) {   // a calibration read-back may still be landing in h_seg_rebound
        if (probe_pending) (void)hipEventSynchronize(ev_probe);
        (void)hipEventDestroy(ev_probe);
    }
    for (hipEvent_t e : ev_call)
        if (e) (void)hipEventDestroy(e);
    for (int i = 0; i < kEvRing; ++i) {
        if (ev_start[i]) (void)hipEventDestroy(ev_start[i]);
        if (ev_stop[i]) (void)hipEventDestroy(ev_stop[i]);
    }
    if (holds_refs)
        for (osk_seg* s : segs) osk::seg_unref(s);
}

void osk::seg_unref(osk_seg* s) {
    if (s && s->refs.fetch_sub(1) == 1) {
        (void)hipSetDevice(s->device);
        delete s;
    }
}

namespace {

int32_t ensure_sq8_seg(osk_seg* s, hipStream_t st);
int32_t ensure_sq8t_seg(osk_seg* s, hipStream_t st, bool wide);
int32_t ensure_split(osk_seg* s, hipStream_t st);
int32_t ensure_sq8(osk_view* v, hipStream_t st);
int32_t ensure_sq8t(osk_view* v, hipStream_t st);
int32_t ensure_sq8w(osk_view* v, hipStream_t st);
int32_t ensure_mfma(osk_view* v, hipStream_t st);

int32_t seg_finish(osk_seg* s, const int32_t* ord_to_doc, hipStream_t st) {
    // row norms
    if (s->enc == ENC_FLOAT32 && s->sim == SIM_COSINE) {
        OSK_HIP(hipMalloc(&s->d_xnorm_f, std::max<int64_t>(1, s->n_rows) * sizeof(float)));
        if (s->n_rows > 0)
            OSK_HIP(launch_row_norms_f32(static_cast<const float4*>(s->d_rows), s->n_rows, s->units,
                                         s->cfg, s->d_xnorm_f, st));
    }
    if (s->enc == ENC_BYTE) {
        OSK_HIP(hipMalloc(&s->d_xnorm_i, std::max<int64_t>(1, s->n_rows) * sizeof(int32_t)));
        if (s->n_rows > 0)
            OSK_HIP(launch_row_norms_i8(static_cast<const int4*>(s->d_rows), s->n_rows, s->units,
                                        s->d_xnorm_i, st));
    }
    if (ord_to_doc) {
        for (int64_t i = 0; i < s->n_rows; ++i) {
            if (ord_to_doc[i] < 0 || ord_to_doc[i] >= s->max_doc ||
                (i > 0 && ord_to_doc[i] <= ord_to_doc[i - 1])) {
                set_error("ord_to_doc must be strictly ascending docIDs in [0, max_doc)");
                return OSK_ERR_INVALID;
            }
        }
        OSK_HIP(hipMalloc(&s->d_ord_to_doc, std::max<int64_t>(1, s->n_rows) * sizeof(int32_t)));
        OSK_HIP(hipMemcpyAsync(s->d_ord_to_doc, ord_to_doc, s->n_rows * sizeof(int32_t),
                               hipMemcpyHostToDevice, st));
    }
    OSK_HIP(hipStreamSynchronize(st));
    // the certified int8 prefilter copy is the default path of float32 searches: built with the segment
    // (staging = the reader's constructor / warmer, S/index/engine/InternalEngine.java:2409-2432), so
    // no search pays for it and the segment's HBM footprint is known at staging
    if (s->enc == ENC_FLOAT32) return ensure_sq8_seg(s, st);
    return OSK_OK;
}

int32_t seg_alloc(int device, int64_t n_rows, int dim, int enc, int sim, int max_doc,
                  const int32_t* ord_to_doc, std::unique_ptr<osk_seg>& out) {
    OSK_REQUIRE(n_rows >= 0, "n_rows must be >= 0");
    OSK_REQUIRE(dim >= 1 && dim <= OSK_MAX_DIM, "dim must be in [1, 4096]");
    OSK_REQUIRE(enc == ENC_FLOAT32 || enc == ENC_BYTE, "unknown encoding");
    OSK_REQUIRE(sim >= 0 && sim <= 3, "unknown similarity");
    OSK_REQUIRE(n_rows <= 0x7FFFFFFFll, "a Lucene segment holds < 2^31 docs");
    if (ord_to_doc == nullptr) OSK_REQUIRE(max_doc >= n_rows, "max_doc < n_rows for a dense field");
    int32_t rc = check_device(device);
    if (rc) return rc;
    auto s = std::make_unique<osk_seg>();
    s->device = device;
    s->n_rows = n_rows;
    s->dim = dim;
    s->enc = enc;
    s->sim = sim;
    s->max_doc = max_doc;
    s->units = units_for(dim, enc);
    s->cfg = cfg_index(s->units);
    const size_t bytes = (size_t)std::max<int64_t>(1, n_rows) * s->units * 16;
    hipError_t e = hipMalloc(&s->d_rows, bytes);
    if (e != hipSuccess) {
        set_error(std::string("hipMalloc of segment rows failed: ") + hipGetErrorString(e));
        return OSK_ERR_OOM;
    }
    out = std::move(s);
    return OSK_OK;
}

}  // namespace

// ------------------------------------------------------------------------------------------------
// C-ABI
// ------------------------------------------------------------------------------------------------
extern "C" {

int32_t osk_abi_version(void) { return OSK_ABI_VERSION; }

int32_t osk_tune_set(const char* key, int64_t value) {
    OSK_GUARD_BEGIN
    OSK_REQUIRE(key != nullptr, "key is null");
    const std::string k(key);
    struct Knob { const char* name; std::atomic<int>* v; int64_t lo, hi; bool testing; };
    const Knob knobs[] = {
        {"scan_nt", &g_tuning.scan_nt, 0, 1, false},
        {"host_batching", &g_tuning.host_batching, 0, 1, false},
        {"host_batch_leaders", &g_tuning.host_batch_leaders, 1, 8, false},
        {"tiles_target", &g_tuning.tiles_target, 0, 1 << 22, false},
        {"tile_slots_per_cu", &g_tuning.tile_slots_per_cu, 1, 64, false},
        {"tile_max_rounds", &g_tuning.tile_max_rounds, 1, 1024, false},
        {"tile_large_slots", &g_tuning.tile_large_slots, 0, 1024, false},
        {"tile_large_slots_512", &g_tuning.tile_large_slots_512, 0, 1024, false},
        {"tile_min_rows", &g_tuning.tile_min_rows, 1, 1 << 24, false},
        {"mfma_min_batch", &g_tuning.mfma_min_batch, 0, 1 << 30, false},
        {"sq8_cost_pct", &g_tuning.sq8_cost_pct, 0, 100000, false},
        {"mfma_units", &g_tuning.mfma_units, 0, 32768, false},
        {"sq8", &g_tuning.sq8, 0, 1, false},
        {"sq6", &g_tuning.sq6, 0, 1, false},
        {"sq6_probe_pct", &g_tuning.sq6_probe_pct, 0, 100, false},
        {"filter_gather", &g_tuning.filter_gather, 0, 1, false},
        {"select_mid_k", &g_tuning.select_mid_k, 0, 1, false},
        {"sel_writer", &g_tuning.sel_writer, 0, 3, false},
        {"gather_min", &g_tuning.gather_min, 0, 1 << 20, false},
        {"sq8_mfma_nt", &g_tuning.sq8_mfma_nt, 0, 1, false},
        {"sq8_mfma_queries", &g_tuning.sq8_mfma_queries, 16, 32, false},
        {"sq8_mfma_min", &g_tuning.sq8_mfma_min, 0, 1 << 20, false},
        {"sq8_wide_min", &g_tuning.sq8_wide_min, 0, 1 << 20, false},
        {"sq8_wide_force", &g_tuning.sq8_wide_force, 0, 1, false},
        {"sq8_wide_phase", &g_tuning.sq8_wide_phase, 0, 1 << 16, false},
        {"sq8_wide_grid", &g_tuning.sq8_wide_grid, 0, 1 << 16, false},
        {"sq8_wide_quarter_rows", &g_tuning.sq8_wide_quarter_rows, 0, 1 << 20, false},
        {"sq8_wide_pilot_rows", &g_tuning.sq8_wide_pilot_rows, 0, 1 << 16, false},
        {"sq8_wide_defer", &g_tuning.sq8_wide_defer, 0, 1, false},
        {"sq8_wide_rows", &g_tuning.sq8_wide_rows, 0, 1, false},
        {"sq8_wide_rows_qcap", &g_tuning.sq8_wide_rows_qcap, 0, 1 << 20, false},
        {"sq8_scan_deep", &g_tuning.sq8_scan_deep, 0, 1, false},
        {"sq8_wide_rows_claim", &g_tuning.sq8_wide_rows_claim, 0, 1, false},
        {"sq6_rebound_stride", &g_tuning.sq6_rebound_stride, 0, 1, false},
        {"sq6_rebound_retest", &g_tuning.sq6_rebound_retest, 0, 1, false},
        {"sq6_rebound_wgs", &g_tuning.sq6_rebound_wgs, 0, 16, false},
        {"sq8_mfma_ring", &g_tuning.sq8_mfma_ring, -1, 8, false},
        {"i8_stream", &g_tuning.i8_stream, 0, 1, false},
        {"call_timing", &g_tuning.call_timing, 0, 1, false},
        {"sq8_mfma_ablate", &g_tuning.sq8_mfma_ablate, 0, 1023, true},   // (also sq6_scan's: 1 no re-bound, 2 no floor,
                                                                          // 16 loads only; sq6_rebound's: 256 no list work)
        {"sq8_force_fallback", &g_tuning.sq8_force_fallback, 0, 1, true},
        {"settle_trace", &g_tuning.settle_trace, 0, 1, true},
        {"mfma_ablate", &g_tuning.mfma_ablate, 0, 255, true},
    };
    for (const Knob& kn : knobs) {
        if (k != kn.name) continue;
#ifndef OSK_TESTING
        if (kn.testing) {
            set_error("tuning key " + k + " exists only in the testing build (libosknn_testing.so)");
            return OSK_ERR_UNSUPPORTED;
        }
#endif
        OSK_REQUIRE(value >= kn.lo && value <= kn.hi, "tuning value out of range for " + k);
        if (k == "sq8_mfma_queries") OSK_REQUIRE(value == 16 || value == 32, "sq8_mfma_queries must be 16 or 32");
        kn.v->store((int)value);
        return OSK_OK;
    }
    set_error("unknown tuning key: " + k);
    return OSK_ERR_INVALID;
    OSK_GUARD_END
}

int32_t osk_testing_glds_probe(int32_t device, int64_t* out_mismatches) {
    OSK_GUARD_BEGIN
    clear_error();
#ifndef OSK_TESTING
    (void)device; (void)out_mismatches;
    set_error("osk_testing_glds_probe exists only in the testing build (libosknn_testing.so)");
    return OSK_ERR_UNSUPPORTED;
#else
    OSK_REQUIRE(out_mismatches != nullptr, "out_mismatches is null");
    int32_t rc = check_device(device);
    if (rc) return rc;
    constexpr int kSrc = 1024, kImg = 1024, kCases = 6;
    std::vector<int4> h_src(kSrc), h_out((size_t)kCases * kImg);
    for (int i = 0; i < kSrc; ++i) h_src[i] = make_int4(i, i ^ 0x5A5A, 3 * i + 1, 7);
    int4 *d_src = nullptr, *d_out = nullptr;
    OSK_HIP(hipMalloc(&d_src, kSrc * sizeof(int4)));
    if (hipMalloc(&d_out, h_out.size() * sizeof(int4)) != hipSuccess) {
        (void)hipFree(d_src);
        set_error("hipMalloc failed");
        return OSK_ERR_DEVICE;
    }
    hipError_t e = hipMemcpy(d_src, h_src.data(), kSrc * sizeof(int4), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = launch_glds_probe(d_src, d_out, nullptr);
    if (e == hipSuccess) e = hipMemcpy(h_out.data(), d_out, h_out.size() * sizeof(int4), hipMemcpyDeviceToHost);
    (void)hipFree(d_src);
    (void)hipFree(d_out);
    if (e != hipSuccess) {
        set_error(std::string("glds probe: ") + hipGetErrorString(e));
        return OSK_ERR_DEVICE;
    }
    // the expected image of each case: DMA k's 64 lanes at 3072 + (N − 1 − k)·2048 + 512 + lane·16, all else −1
    int64_t bad = 0;
    const int ns[kCases] = {1, 2, 4, 1, 2, 4}, gs[kCases] = {1024, 1024, 1024, kAuxGroupF4 * 16, kAuxGroupF4 * 16,
                                                             kAuxGroupF4 * 16};
    for (int c = 0; c < kCases; ++c) {
        std::vector<int4> want(kImg, make_int4(-1, -1, -1, -1));
        for (int k = 0; k < ns[c]; ++k)
            for (int l = 0; l < 64; ++l) want[(3072 + (ns[c] - 1 - k) * 2048 + 512) / 16 + l] = h_src[(k * gs[c]) / 16 + l];
        for (int i = 0; i < kImg; ++i) {
            const int4 a = h_out[(size_t)c * kImg + i], b = want[i];
            bad += a.x != b.x || a.y != b.y || a.z != b.z || a.w != b.w;
        }
    }
    *out_mismatches = bad;
    return OSK_OK;
#endif
    OSK_GUARD_END
}

int32_t osk_device_count(int32_t* n) {
    OSK_GUARD_BEGIN
    OSK_REQUIRE(n != nullptr, "n is null");
    *n = device_count_cached();
    return OSK_OK;
    OSK_GUARD_END
}

int32_t osk_seg_stage(int32_t device, const void* rows, int64_t n_rows, int32_t dim,
                      int32_t encoding, int32_t similarity, const int32_t* ord_to_doc,
                      int32_t max_doc, osk_seg** out) {
    OSK_GUARD_BEGIN
    clear_error();
    OSK_REQUIRE(out != nullptr, "out is null");
    OSK_REQUIRE(rows != nullptr || n_rows == 0, "rows is null");
    std::unique_ptr<osk_seg> s;
    int32_t rc = seg_alloc(device, n_rows, dim, encoding, similarity, max_doc, ord_to_doc, s);
    if (rc) return rc;
    hipStream_t st = device_stream(device);
    const int64_t elem = encoding == ENC_FLOAT32 ? 4 : 1;
    const int64_t src_pitch = (int64_t)dim * elem;
    const int64_t dst_pitch = (int64_t)s->units * 16;
    if (n_rows > 0) {
        OSK_HIP(hipMemset2DAsync(s->d_rows, dst_pitch, 0, dst_pitch, n_rows, st));
        OSK_HIP(hipMemcpy2DAsync(s->d_rows, dst_pitch, rows, src_pitch, src_pitch, n_rows,
                                 hipMemcpyHostToDevice, st));
    }
    rc = seg_finish(s.get(), ord_to_doc, st);
    if (rc) return rc;
    *out = s.release();
    return OSK_OK;
    OSK_GUARD_END
}

int32_t osk_seg_stage_file(int32_t device, const char* path, int64_t data_offset, int64_t n_rows, int32_t dim,
                           int32_t encoding, int32_t similarity, const int32_t* ord_to_doc, int32_t max_doc,
                           osk_seg** out) {
    OSK_GUARD_BEGIN
    clear_error();
    OSK_REQUIRE(out != nullptr && path != nullptr, "null argument");
    OSK_REQUIRE(data_offset >= 0, "negative data offset");
    std::unique_ptr<osk_seg> s;
    int32_t rc = seg_alloc(device, n_rows, dim, encoding, similarity, max_doc, ord_to_doc, s);
    if (rc) return rc;
    hipStream_t st = device_stream(device);
    const int64_t row_bytes = (int64_t)dim * (encoding == ENC_FLOAT32 ? 4 : 1);
    const int64_t bytes = n_rows * row_bytes;
    const int64_t dst_pitch = (int64_t)s->units * 16;
    if (n_rows > 0) {
        // the .vec slice: memory-mapped (as FsDirectoryFactory maps .vec under hybridfs), copied chunk by
        // chunk into one of two pinned buffers while the other one's H2D copy runs, then into the
        // segment's padded rows (zeros past dim)
        const int fd = ::open(path, O_RDONLY | O_CLOEXEC);
        if (fd < 0) {
            set_error(std::string("cannot open ") + path + ": " + std::strerror(errno));
            return OSK_ERR_INVALID;
        }
        struct stat sb;
        if (::fstat(fd, &sb) != 0 || sb.st_size < data_offset + bytes) {
            ::close(fd);
            set_error(std::string(path) + " is shorter than the field's vector data");
            return OSK_ERR_INVALID;
        }
        const int64_t page = ::sysconf(_SC_PAGESIZE);
        const int64_t map_off = data_offset / page * page;
        const size_t map_len = (size_t)(data_offset + bytes - map_off);
        void* map = ::mmap(nullptr, map_len, PROT_READ, MAP_PRIVATE, fd, map_off);
        ::close(fd);
        if (map == MAP_FAILED) {
            set_error(std::string("mmap of ") + path + " failed: " + std::strerror(errno));
            return OSK_ERR_INVALID;
        }
        (void)::madvise(map, map_len, MADV_SEQUENTIAL);
        const char* src = static_cast<const char*>(map) + (data_offset - map_off);
        constexpr int64_t kChunk = 32ll << 20;
        const int64_t rows_per = std::max<int64_t>(1, kChunk / row_bytes);
        HostPinned ring[2];
        hipEvent_t ev[2] = {nullptr, nullptr};
        bool used[2] = {false, false};
        int32_t err = OSK_OK;
        auto fail = [&](hipError_t e, const char* what) {
            set_error(std::string(what) + ": " + hipGetErrorString(e));
            err = OSK_ERR_DEVICE;
        };
        hipError_t e;
        for (int i = 0; i < 2 && !err; ++i) {
            if ((e = ring[i].reserve((size_t)std::min(n_rows, rows_per) * row_bytes)) != hipSuccess) fail(e, "pinned staging buffer");
            else if ((e = hipEventCreateWithFlags(&ev[i], hipEventDisableTiming)) != hipSuccess) fail(e, "staging event");
        }
        if (!err && (e = hipMemset2DAsync(s->d_rows, dst_pitch, 0, dst_pitch, n_rows, st)) != hipSuccess)
            fail(e, "hipMemset2DAsync");
        int slot = 0;
        for (int64_t r0 = 0; r0 < n_rows && !err; r0 += rows_per, slot ^= 1) {
            const int64_t cnt = std::min(rows_per, n_rows - r0);
            if (used[slot] && (e = hipEventSynchronize(ev[slot])) != hipSuccess) { fail(e, "hipEventSynchronize"); break; }
            std::memcpy(ring[slot].p, src + r0 * row_bytes, (size_t)(cnt * row_bytes));
            if ((e = hipMemcpy2DAsync(static_cast<char*>(s->d_rows) + r0 * dst_pitch, dst_pitch, ring[slot].p, row_bytes,
                                      row_bytes, cnt, hipMemcpyHostToDevice, st)) != hipSuccess) { fail(e, "hipMemcpy2DAsync"); break; }
            if ((e = hipEventRecord(ev[slot], st)) != hipSuccess) { fail(e, "hipEventRecord"); break; }
            used[slot] = true;
        }
        if ((e = hipStreamSynchronize(st)) != hipSuccess && !err) fail(e, "hipStreamSynchronize");
        for (int i = 0; i < 2; ++i)
            if (ev[i]) (void)hipEventDestroy(ev[i]);
        ::munmap(map, map_len);
        if (err) return err;
    }
    rc = seg_finish(s.get(), ord_to_doc, st);
    if (rc) return rc;
    *out = s.release();
    return OSK_OK;
    OSK_GUARD_END
}

int32_t osk_seg_stage_device(int32_t device, const void* d_rows, int64_t src_pitch_bytes,
                             int64_t n_rows, int32_t dim, int32_t encoding, int32_t similarity,
                             const int32_t* ord_to_doc, int32_t max_doc, osk_seg** out) {
    OSK_GUARD_BEGIN
    clear_error();
    OSK_REQUIRE(out != nullptr, "out is null");
    OSK_REQUIRE(d_rows != nullptr || n_rows == 0, "d_rows is null");
    std::unique_ptr<osk_seg> s;
    int32_t rc = seg_alloc(device, n_rows, dim, encoding, similarity, max_doc, ord_to_doc, s);
    if (rc) return rc;
    hipStream_t st = device_stream(device);
    const int64_t elem = encoding == ENC_FLOAT32 ? 4 : 1;
    OSK_REQUIRE(src_pitch_bytes >= (int64_t)dim * elem, "src_pitch_bytes < dim * element size");
    if (n_rows > 0)
        OSK_HIP(launch_pad_rows(d_rows, src_pitch_bytes, s->d_rows, (int64_t)s->units * 16, n_rows,
                                (int64_t)dim * elem, st));
    rc = seg_finish(s.get(), ord_to_doc, st);
    if (rc) return rc;
    *out = s.release();
    return OSK_OK;
    OSK_GUARD_END
}

int32_t osk_seg_synth(int32_t device, int64_t n_rows, int32_t dim, int32_t encoding,
                      int32_t similarity, uint64_t seed, int32_t dist, int64_t row0,
                      osk_seg** out) {
    OSK_GUARD_BEGIN
    clear_error();
    OSK_REQUIRE(out != nullptr, "out is null");
    OSK_REQUIRE(dist >= 0 && dist <= 4, "unknown dist");
    OSK_REQUIRE((dist == DIST_INT8) == (encoding == ENC_BYTE), "dist INT8 <=> encoding BYTE");
    OSK_REQUIRE(n_rows <= 0x7FFFFFFFll, "a Lucene segment holds < 2^31 docs");
    std::unique_ptr<osk_seg> s;
    int32_t rc = seg_alloc(device, n_rows, dim, encoding, similarity, (int32_t)n_rows, nullptr, s);
    if (rc) return rc;
    hipStream_t st = device_stream(device);
    if (n_rows > 0)
        OSK_HIP(launch_synth(s->d_rows, n_rows, dim, s->units, encoding, seed, dist, row0, st));
    rc = seg_finish(s.get(), nullptr, st);
    if (rc) return rc;
    *out = s.release();
    return OSK_OK;
    OSK_GUARD_END
}

int32_t osk_seg_release(osk_seg* seg) {
    OSK_GUARD_BEGIN
    if (!seg) return OSK_OK;
    seg_unref(seg);   // freed when no view holds it any more
    return OSK_OK;
    OSK_GUARD_END
}

int32_t osk_seg_retain(osk_seg* seg) {
    OSK_GUARD_BEGIN
    OSK_REQUIRE(seg != nullptr, "seg is null");
    seg->refs.fetch_add(1);
    return OSK_OK;
    OSK_GUARD_END
}

int32_t osk_seg_footprint(const osk_seg* seg, int64_t* hbm_bytes) {
    OSK_GUARD_BEGIN
    OSK_REQUIRE(seg != nullptr && hbm_bytes != nullptr, "null argument");
    *hbm_bytes = seg->hbm_bytes();
    return OSK_OK;
    OSK_GUARD_END
}

int32_t osk_seg_warm(osk_seg* seg, int32_t what) {
    OSK_GUARD_BEGIN
    clear_error();
    OSK_REQUIRE(seg != nullptr, "seg is null");
    OSK_REQUIRE((what & ~OSK_WARM_ALL) == 0, "unknown warm flags");
    int32_t rc = check_device(seg->device);
    if (rc) return rc;
    if (seg->enc != ENC_FLOAT32) return OSK_OK;   // byte fields scan their rows directly
    hipStream_t st = device_stream(seg->device);
    if (what & (OSK_WARM_PREFILTER | OSK_WARM_PREFILTER_MFMA)) {
        rc = ensure_sq8_seg(seg, st);
        if (rc) return rc;
    }
    if ((what & OSK_WARM_PREFILTER_MFMA) && sq8_mfma_supported((seg->dim + 15) / 16)) {
        rc = ensure_sq8t_seg(seg, st, false);
        if (rc) return rc;
    }
    if (what & OSK_WARM_BATCHED) return ensure_split(seg, st);
    return OSK_OK;
    OSK_GUARD_END
}

int32_t osk_seg_info(const osk_seg* seg, int64_t* n_rows, int32_t* dim, int32_t* encoding,
                     int32_t* similarity, int32_t* max_doc, int32_t* device) {
    OSK_GUARD_BEGIN
    OSK_REQUIRE(seg != nullptr, "seg is null");
    if (n_rows) *n_rows = seg->n_rows;
    if (dim) *dim = seg->dim;
    if (encoding) *encoding = seg->enc;
    if (similarity) *similarity = seg->sim;
    if (max_doc) *max_doc = seg->max_doc;
    if (device) *device = seg->device;
    return OSK_OK;
    OSK_GUARD_END
}

int32_t osk_view_create(osk_seg* const* segs, int32_t n_segs, const int32_t* seg_shard,
                        const int32_t* seg_doc_base, int32_t n_shards, const int32_t* shard_index,
                        osk_view** out) {
    OSK_GUARD_BEGIN
    clear_error();
    OSK_REQUIRE(out != nullptr && segs != nullptr, "null argument");
    OSK_REQUIRE(n_segs >= 1, "need at least one segment");
    OSK_REQUIRE(n_shards >= 1, "need at least one shard");
    const osk_seg* s0 = segs[0];
    OSK_REQUIRE(s0 != nullptr, "null segment");
    for (int i = 0; i < n_segs; ++i) {
        OSK_REQUIRE(segs[i] != nullptr, "null segment");
        OSK_REQUIRE(segs[i]->device == s0->device && segs[i]->dim == s0->dim &&
                        segs[i]->enc == s0->enc && segs[i]->sim == s0->sim,
                    "segments of a view must share device, dim, encoding and similarity");
        const int sh = seg_shard ? seg_shard[i] : 0;
        OSK_REQUIRE(sh >= 0 && sh < n_shards, "seg_shard out of range");
        OSK_REQUIRE(!seg_doc_base || seg_doc_base[i] >= 0, "negative doc base");
    }
    int32_t rc = check_device(s0->device);
    if (rc) return rc;
    auto v = std::make_unique<osk_view>();
    v->device = s0->device;
    v->dim = s0->dim;
    v->enc = s0->enc;
    v->sim = s0->sim;
    v->units = s0->units;
    v->cfg = s0->cfg;
    v->segs.assign(segs, segs + n_segs);
    v->seg_shard.resize(n_segs);
    for (int i = 0; i < n_segs; ++i) v->seg_shard[i] = seg_shard ? seg_shard[i] : 0;
    v->n_shards = n_shards;
    v->shard_index.resize(n_shards);
    for (int s = 0; s < n_shards; ++s) v->shard_index[s] = shard_index ? shard_index[s] : s;

    // tiles: a whole number of "rounds" of the chip's resident workgroup slots (CUs × tile_slots_per_cu;
    // the scan kernels run 4 waves/SIMD = 4 workgroups of 256 threads per CU), so every round is full
    // and no tail round runs with most slots idle (profiles/r01e/tiles_ab.txt: 1.25M rows, 1024 tiles
    // 0.190 ms vs 1221 tiles 0.219 ms).  Rounds grow with the view up to tile_max_rounds; a tile never
    // drops below 8 row-groups per wave nor tile_min_rows rows.
    static const int kL[9] = {4, 8, 8, 16, 16, 16, 32, 64, 64};
    const int R = 64 / kL[v->cfg];
    int64_t total = 0;
    for (int i = 0; i < n_segs; ++i) total += segs[i]->n_rows;
    int64_t min_rows = std::max<int64_t>(4LL * R * 8, (int)g_tuning.tile_min_rows);
    int64_t target = g_tuning.tiles_target;
    if (target <= 0) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, s0->device) != hipSuccess || cus <= 0)
            cus = 256;
        const int64_t slots = (int64_t)cus * std::max(1, (int)g_tuning.tile_slots_per_cu);
        const int64_t rounds = std::min<int64_t>(std::max(1, (int)g_tuning.tile_max_rounds),
                                                 std::max<int64_t>(1, total / (slots * min_rows)));
        target = rounds * slots;
        // large views: whole rounds of BOTH scan kernels' residency.  sq8_scan holds 4 workgroups per
        // CU but sq8_mfma at 32 queries only 3 (LDS), so 4 rounds of 4 slots leave sq8_mfma a third
        // of a tail round.  cus × tile_large_slots tiles (24 = 2 · lcm(3, 4)) are 6 full sq8_scan rounds
        // and 8 full sq8_mfma rounds (profiles/r01l/tiles_ab.txt: C3 b32 2.72 -> 2.47 ms, C4 b32
        // 7.2 -> 6.5 ms, C3 b1 within 1%).
        // Rows of ≥ 512 dims (the 6-bit tier's views, C3/C5i-shaped) take half as many (12 = lcm(3, 4): 3 full
        // sq8_scan rounds, 4 sq8_mfma rounds): their tiles are heavy enough that fewer, fuller workgroups win —
        // the 6-bit tier's pilot, re-bound and settle run over fewer lists (C3 b1 +2.0 % at 4 in flight and one
        // in flight, 3 interleaved A/B pairs, profiles/r05m/), C3 b32 and C5i gained too; C4 b32 (96 dims)
        // lost 9 % with 12 (profiles/r05j/), so lighter rows keep tile_large_slots.
        const int slots_large = v->dim >= 512 ? (int)g_tuning.tile_large_slots_512 : (int)g_tuning.tile_large_slots;
        const int64_t large = (int64_t)cus * slots_large;
        if (slots_large > 0 && total >= large * min_rows) target = large;
        // views smaller than one round at tile_min_rows (C1: 100k rows): latency-bound, so spread them
        // over more of the chip with tiles down to 8 row groups per wave (≥ 256 rows): C1's scan
        // 34 -> 16 µs (profiles/r02o/tile_min_rows.txt); a full round is unaffected (C2: 1024 tiles)
        if (total < slots * min_rows) min_rows = std::max<int64_t>(4LL * R * 8, 256);
    }
    // split the target over segments in proportion to their rows (largest remainder), each segment's
    // share capped so its tiles keep ≥ min_rows rows
    std::vector<int64_t> seg_tiles(n_segs, 0);
    {
        int64_t given = 0;
        std::vector<std::pair<double, int>> rem;
        for (int i = 0; i < n_segs; ++i) {
            const int64_t n = segs[i]->n_rows;
            if (n == 0) continue;
            const double share = total > 0 ? (double)n * (double)target / (double)total : 1.0;
            const int64_t cap = std::max<int64_t>(1, (n + min_rows - 1) / min_rows);
            seg_tiles[i] = std::min<int64_t>(cap, std::max<int64_t>(1, (int64_t)share));
            given += seg_tiles[i];
            rem.push_back({share - (double)(int64_t)share, i});
        }
        std::sort(rem.begin(), rem.end(), [](auto& a, auto& b) { return a.first > b.first || (a.first == b.first && a.second < b.second); });
        for (size_t j = 0; j < rem.size() && given < target; ++j) {
            const int i = rem[j].second;
            const int64_t cap = std::max<int64_t>(1, (segs[i]->n_rows + min_rows - 1) / min_rows);
            if (seg_tiles[i] < cap) { ++seg_tiles[i]; ++given; }
        }
    }
    std::vector<TileDev> tiles;
    v->shard_tile_begin.assign(n_shards + 1, 0);
    for (int sh = 0; sh < n_shards; ++sh) {
        v->shard_tile_begin[sh] = (int32_t)tiles.size();
        for (int i = 0; i < n_segs; ++i) {
            if ((seg_shard ? seg_shard[i] : 0) != sh) continue;
            const int64_t n = segs[i]->n_rows;
            if (n == 0) continue;
            const int64_t nt = seg_tiles[i];
            // balanced split at multiples of 16 rows (sq8_mfma's row groups then start on its tiled
            // copy's 16-row blocks): tile t = rows [⌊n·t/nt⌋₁₆, ⌊n·(t+1)/nt⌋₁₆), the last one ends at n
            auto cut = [&](int64_t t) { return t >= nt ? n : (n * t / nt) & ~(int64_t)15; };
            for (int64_t t = 0; t < nt; ++t)
                if (cut(t + 1) > cut(t)) tiles.push_back(TileDev{i, sh, cut(t), cut(t + 1)});
        }
    }
    v->shard_tile_begin[n_shards] = (int32_t)tiles.size();
    v->n_tiles = (int)tiles.size();
    // each tile's first row's slot in its shard's candidate region (the select path's collect)
    std::vector<int32_t> tile_coff(std::max<size_t>(1, tiles.size()), 0);
    for (int sh = 0; sh < n_shards; ++sh) {
        int64_t acc = 0;
        for (int t = v->shard_tile_begin[sh]; t < v->shard_tile_begin[sh + 1]; ++t) {
            tile_coff[t] = (int32_t)std::min<int64_t>(acc, INT32_MAX);
            acc += tiles[t].row_end - tiles[t].row_begin;
        }
    }
    OSK_REQUIRE(v->n_tiles < (1 << 24), "too many tiles");
    // dispatch order of the 6-bit scan: tiles interleaved over shards (shard s's j-th of n_s tiles at
    // ≈ (j + ½)/n_s of the grid), so every round of resident workgroups scans a slice of every shard and
    // each shard's floor rises from the first round on (osk_sq6.hip)
    std::vector<int32_t> tile_order(std::max<size_t>(1, tiles.size()), 0);
    {
        std::vector<std::pair<double, int>> key;
        for (int sh = 0; sh < n_shards; ++sh) {
            const int t0 = v->shard_tile_begin[sh], n = v->shard_tile_begin[sh + 1] - t0;
            for (int j = 0; j < n; ++j) key.push_back({(j + 0.5) / n, t0 + j});
        }
        std::stable_sort(key.begin(), key.end(), [](auto& a, auto& b) { return a.first < b.first; });
        for (size_t i = 0; i < key.size(); ++i) tile_order[i] = key[i].second;
    }

    v->seg_doc_base.resize(n_segs);
    for (int i = 0; i < n_segs; ++i) v->seg_doc_base[i] = seg_doc_base ? seg_doc_base[i] : 0;
    std::vector<int64_t> vrow(n_segs);   // view-global row of each segment's ord 0
    int64_t vacc = 0;
    for (int i = 0; i < n_segs; ++i) {
        vrow[i] = vacc;
        vacc += segs[i]->n_rows;
    }
    OSK_REQUIRE(total < 0xFFFFFFFFll, "a view holds < 2^32 rows");
    std::vector<SegDev> sd = seg_devs(v.get());
    hipStream_t st = device_stream(v->device);
    OSK_HIP(v->d_segs.reserve(sizeof(SegDev) * n_segs));
    OSK_HIP(v->d_tiles.reserve(sizeof(TileDev) * std::max<size_t>(1, tiles.size())));
    OSK_HIP(v->d_shard_tile_begin.reserve(sizeof(int32_t) * (n_shards + 1)));
    OSK_HIP(v->d_shard_index.reserve(sizeof(int32_t) * n_shards));
    OSK_HIP(v->d_tile_coff.reserve(sizeof(int32_t) * tile_coff.size()));
    OSK_HIP(v->d_tile_order.reserve(sizeof(int32_t) * tile_order.size()));
    OSK_HIP(v->d_seg_vrow.reserve(sizeof(int64_t) * n_segs));
    OSK_HIP(v->d_counters.reserve(sizeof(unsigned long long) * 24));
    OSK_HIP(hipMemsetAsync(v->d_counters.p, 0, sizeof(unsigned long long) * 24, st));
    OSK_HIP(hipMemcpyAsync(v->d_seg_vrow.p, vrow.data(), sizeof(int64_t) * n_segs, hipMemcpyHostToDevice, st));
    OSK_HIP(hipMemcpyAsync(v->d_segs.p, sd.data(), sizeof(SegDev) * n_segs, hipMemcpyHostToDevice, st));
    if (!tiles.empty())
        OSK_HIP(hipMemcpyAsync(v->d_tiles.p, tiles.data(), sizeof(TileDev) * tiles.size(),
                               hipMemcpyHostToDevice, st));
    OSK_HIP(hipMemcpyAsync(v->d_shard_tile_begin.p, v->shard_tile_begin.data(),
                           sizeof(int32_t) * (n_shards + 1), hipMemcpyHostToDevice, st));
    OSK_HIP(hipMemcpyAsync(v->d_shard_index.p, v->shard_index.data(), sizeof(int32_t) * n_shards,
                           hipMemcpyHostToDevice, st));
    OSK_HIP(hipMemcpyAsync(v->d_tile_coff.p, tile_coff.data(), sizeof(int32_t) * tile_coff.size(),
                           hipMemcpyHostToDevice, st));
    OSK_HIP(hipMemcpyAsync(v->d_tile_order.p, tile_order.data(), sizeof(int32_t) * tile_order.size(),
                           hipMemcpyHostToDevice, st));
    OSK_HIP(hipStreamSynchronize(st));
    for (osk_seg* sg : v->segs) sg->refs.fetch_add(1);   // released by ~osk_view
    *out = v.release();
    return OSK_OK;
    OSK_GUARD_END
}

int32_t osk_view_warm(osk_view* view, int32_t what) {
    OSK_GUARD_BEGIN
    clear_error();
    OSK_REQUIRE(view != nullptr, "view is null");
    OSK_REQUIRE((what & ~OSK_WARM_ALL) == 0, "unknown warm flags");
    for (osk_seg* s : view->segs) {
        int32_t rc = osk_seg_warm(s, what);
        if (rc) return rc;
    }
    if (view->enc != ENC_FLOAT32 || view->n_tiles == 0) return OSK_OK;
    int32_t rc = check_device(view->device);
    if (rc) return rc;
    hipStream_t st = device_stream(view->device);
    std::lock_guard<std::mutex> lk(view->mu);
    rc = order_after_last(view, st);
    if (rc) return rc;
    if (what & (OSK_WARM_PREFILTER | OSK_WARM_PREFILTER_MFMA)) {
        rc = ensure_sq8(view, st);
        if (rc) return rc;
    }
    if ((what & OSK_WARM_PREFILTER_MFMA) && sq8_mfma_supported((view->dim + 15) / 16)) {
        rc = ensure_sq8t(view, st);
        if (rc) return rc;
    }
    if (what & OSK_WARM_BATCHED) return ensure_mfma(view, st);
    return OSK_OK;
    OSK_GUARD_END
}

int32_t osk_view_release(osk_view* view) {
    OSK_GUARD_BEGIN
    if (!view) return OSK_OK;
    (void)hipSetDevice(view->device);
    delete view;
    return OSK_OK;
    OSK_GUARD_END
}

}  // extern "C"

namespace {

// Scan-kernel timing (osk_view_profile).  The streaming and prefilter scans stamp v->ev0 / v->ev1
// from their own dispatch packets (first and last launch of the call: launch_ev); the MFMA path,
// several launches, brackets them with event records (record = true).
int32_t profile_fold(osk_view* v, int slot) {
    if (!v->ev_pending[slot]) return OSK_OK;
    float ms = 0.f;
    OSK_HIP(hipEventSynchronize(v->ev_stop[slot]));
    OSK_HIP(hipEventElapsedTime(&ms, v->ev_start[slot], v->ev_stop[slot]));
    v->scan_ms += ms;
    v->scan_calls += 1;
    v->ev_pending[slot] = false;
    return OSK_OK;
}

int32_t profile_begin(osk_view* v, hipStream_t st, bool record) {
    const int slot = (int)(v->ev_next++ % osk_view::kEvRing);
    int32_t rc = profile_fold(v, slot);   // the call kEvRing calls ago
    if (rc) return rc;
    v->ev0 = v->ev_start[slot];
    v->ev1 = v->ev_stop[slot];
    v->ev_pending[slot] = false;
    if (record) OSK_HIP(hipEventRecord(v->ev0, st));
    return OSK_OK;
}

int32_t profile_end(osk_view* v, hipStream_t st, bool record) {
    if (!v->profile) return OSK_OK;
    if (record) OSK_HIP(hipEventRecord(v->ev1, st));
    v->ev_pending[(v->ev_next - 1) % osk_view::kEvRing] = true;
    return OSK_OK;
}

// (start, stop) events for launch q0 of a call that launches [0, nq) in chunks of kMaxNQ
inline hipEvent_t launch_ev_start(const osk_view* v, int q0) { return v->profile && q0 == 0 ? v->ev0 : nullptr; }
inline hipEvent_t launch_ev_stop(const osk_view* v, int q0, int nq) {
    return v->profile && q0 + kMaxNQ >= nq ? v->ev1 : nullptr;
}

// Streaming exact scan of queries already in the padded unit layout (≤ 8 per launch) + per-shard merge.
int32_t stream_search(osk_view* v, const void* qpad, const void* qnorm, int nq, int k, int UP,
                      const uint64_t* const* d_accept, uint64_t* d_shard_keys, int32_t* d_shard_counts,
                      int64_t* d_visited, hipStream_t st) {
    OSK_HIP(v->ws_cand.reserve(sizeof(uint64_t) * (size_t)nq * v->n_tiles * k));
    ScanParams p{};
    p.segs = v->d_segs.as<SegDev>();
    p.tiles = v->d_tiles.as<TileDev>();
    p.accept = d_accept;
    p.cand = v->ws_cand.as<uint64_t>();
    p.visited = reinterpret_cast<unsigned long long*>(d_visited);
    p.n_tiles = v->n_tiles;
    p.units = v->units;
    p.k = k;
    p.sim = v->sim;
    p.dim = v->dim;
    for (int q0 = 0; q0 < nq; q0 += kMaxNQ) {
        const int qc = std::min(kMaxNQ, nq - q0);
        p.q0 = q0;
        p.q_count = qc;
        p.q = static_cast<const char*>(qpad) + (size_t)q0 * UP * 16;
        p.qnorm_f = static_cast<const float*>(qnorm) + q0;
        p.qnorm_i = static_cast<const int32_t*>(qnorm) + q0;
        OSK_HIP(launch_scan(v->enc, v->cfg, qc, p, st, launch_ev_start(v, q0), launch_ev_stop(v, q0, nq)));
    }
    int32_t rc = profile_end(v, st, false);
    if (rc) return rc;
    OSK_HIP(launch_merge_shards(v->ws_cand.as<uint64_t>(), v->n_tiles,
                                v->d_shard_tile_begin.as<int32_t>(), v->n_shards, nq, k,
                                d_shard_keys, d_shard_counts, st));
    return OSK_OK;
}

// The segment's bf16 hi/lo copy in MFMA fragment order (+ |x|² rows and their max).  Built once.
int32_t ensure_split(osk_seg* s, hipStream_t st) {
    std::lock_guard<std::mutex> lk(s->mu);
    if (s->d_split) return OSK_OK;
    const int KS = ((s->units + 7) / 8 + kKsAlign - 1) / kKsAlign * kKsAlign;   // 32-dim K-steps (padded)
    const int64_t n_tiles = (s->n_rows + 127) / 128;        // 128-row tiles
    const int64_t n_rb = std::max<int64_t>(1, n_tiles) * 8;
    if (!s->d_xnorm_f) {
        OSK_HIP(hipMalloc(&s->d_xnorm_f, std::max<int64_t>(1, s->n_rows) * sizeof(float)));
        if (s->n_rows > 0)
            OSK_HIP(launch_row_norms_f32(static_cast<const float4*>(s->d_rows), s->n_rows, s->units, s->cfg,
                                         s->d_xnorm_f, st));
    }
    void* split = nullptr;
    hipError_t e = hipMalloc(&split, (size_t)n_rb * KS * 2 * 1024);
    if (e != hipSuccess) {
        set_error(std::string("hipMalloc of the MFMA split copy failed: ") + hipGetErrorString(e));
        return OSK_ERR_OOM;
    }
    OSK_HIP(launch_split_rows(static_cast<const float4*>(s->d_rows), s->n_rows, s->units, KS, n_rb, split, st));
    OSK_HIP(hipMalloc(&s->d_xsqrt, std::max<int64_t>(1, s->n_rows) * sizeof(float)));
    if (s->n_rows > 0) OSK_HIP(launch_row_sqrt(s->d_xnorm_f, s->n_rows, s->d_xsqrt, st));
    OSK_HIP(hipMalloc(&s->d_maxnorm2, sizeof(unsigned)));
    OSK_HIP(hipMemsetAsync(s->d_maxnorm2, 0, sizeof(unsigned), st));
    if (s->n_rows > 0) OSK_HIP(launch_max_norm2(s->d_xnorm_f, s->n_rows, s->d_maxnorm2, st));
    unsigned bits = 0;
    OSK_HIP(hipMemcpyAsync(&bits, s->d_maxnorm2, sizeof(unsigned), hipMemcpyDeviceToHost, st));
    OSK_HIP(hipStreamSynchronize(st));
    std::memcpy(&s->h_maxnorm2, &bits, 4);
    s->d_split = split;
    s->split_KS = KS;
    return OSK_OK;
}

// MFMA work units (runs of 128-row tiles, contiguous per shard) and per-shard bounds.  Built once.
int32_t ensure_mfma(osk_view* v, hipStream_t st) {
    if (v->mfma_ready) return OSK_OK;
    const int ns = (int)v->segs.size();
    std::vector<const void*> splits(ns);
    std::vector<const float*> xsq(ns);
    std::vector<int64_t> vrow(ns);
    int64_t acc = 0, total_tiles = 0;
    for (int i = 0; i < ns; ++i) {
        int32_t rc = ensure_split(v->segs[i], st);
        if (rc) return rc;
        splits[i] = v->segs[i]->d_split;
        xsq[i] = v->segs[i]->d_xsqrt;
        vrow[i] = acc;
        acc += v->segs[i]->n_rows;
        total_tiles += (v->segs[i]->n_rows + 127) / 128;
    }
    OSK_REQUIRE(acc < 0xFFFFFFFFll, "a view holds < 2^32 rows");
    {   // ensure_split may have added row norms: refresh the device segment table
        const std::vector<SegDev> sd = seg_devs(v);
        OSK_HIP(hipMemcpyAsync(v->d_segs.p, sd.data(), sizeof(SegDev) * sd.size(), hipMemcpyHostToDevice, st));
    }
    // auto: one workgroup per CU (1 per CU fits: 255 VGPRs, 143 KiB LDS) in 1 round below 16k tiles
    // (C2 b256: 0.74 → 0.65 ms, fewer pilot tiles), else 2 rounds (C3 b256: 11.6 ms against 11.7;
    // 384 units, 1.5 rounds, lose 30 %; profiles/r02q/mfma_units.txt)
    const int64_t target = g_tuning.mfma_units > 0 ? (int64_t)g_tuning.mfma_units : (total_tiles < 16384 ? 256 : 512);
    const int64_t per = std::max<int64_t>(1, (total_tiles + target - 1) / target);
    std::vector<MfmaUnit> units;
    std::vector<int32_t> shard_list_begin(v->n_shards + 1, 0);
    std::vector<float> shard_max(v->n_shards, 0.0f);
    for (int sh = 0; sh < v->n_shards; ++sh) {
        shard_list_begin[sh] = (int32_t)units.size() * 2;
        for (int i = 0; i < ns; ++i) {
            if (v->seg_shard[i] != sh) continue;
            shard_max[sh] = std::max(shard_max[sh], v->segs[i]->h_maxnorm2);
            const int64_t nt = (v->segs[i]->n_rows + 127) / 128;
            for (int64_t t = 0; t < nt; t += per)
                units.push_back(MfmaUnit{i, sh, t, std::min(nt, t + per), vrow[i]});
        }
    }
    shard_list_begin[v->n_shards] = (int32_t)units.size() * 2;
    v->n_munits = (int)units.size();
    OSK_REQUIRE(v->n_munits > 0 && v->n_munits < 65536, "bad MFMA unit count");
    v->mfma_KS = ((v->units + 7) / 8 + kKsAlign - 1) / kKsAlign * kKsAlign;
    // |Σ approx − Σ device order| ≤ c·|x||q|: bf16 split (3·2^-16) + fp32 accumulation of the
    // 3·Kpad MFMA products and of the Kpad device-order products (γ_n ≈ n·2^-24), ×1.5 margin.
    const double kpad = 32.0 * v->mfma_KS;
    v->mfma_c = 1.5 * (3.0 * std::ldexp(1.0, -16) + 4.0 * kpad * std::ldexp(1.0, -24));
    OSK_HIP(v->d_munits.reserve(sizeof(MfmaUnit) * units.size()));
    OSK_HIP(v->d_seg_split.reserve(sizeof(void*) * ns));
    OSK_HIP(v->d_seg_xsqrt.reserve(sizeof(void*) * ns));
    OSK_HIP(v->d_shard_unit_begin.reserve(sizeof(int32_t) * (v->n_shards + 1)));
    OSK_HIP(v->d_shard_maxnorm2.reserve(sizeof(float) * v->n_shards));
    OSK_HIP(hipMemcpyAsync(v->d_munits.p, units.data(), sizeof(MfmaUnit) * units.size(), hipMemcpyHostToDevice, st));
    OSK_HIP(hipMemcpyAsync(v->d_seg_split.p, splits.data(), sizeof(void*) * ns, hipMemcpyHostToDevice, st));
    OSK_HIP(hipMemcpyAsync(v->d_seg_xsqrt.p, xsq.data(), sizeof(void*) * ns, hipMemcpyHostToDevice, st));
    OSK_HIP(hipMemcpyAsync(v->d_shard_unit_begin.p, shard_list_begin.data(), sizeof(int32_t) * (v->n_shards + 1),
                           hipMemcpyHostToDevice, st));
    OSK_HIP(hipMemcpyAsync(v->d_shard_maxnorm2.p, shard_max.data(), sizeof(float) * v->n_shards,
                           hipMemcpyHostToDevice, st));
    OSK_HIP(hipStreamSynchronize(st));
    v->mfma_ready = true;
    return OSK_OK;
}

// Batched search: MFMA candidates → per-shard approx top-k' → exact re-score + certificate →
// exact streaming scan for any query whose certificate failed.  ws_q / ws_qnorm hold the padded
// queries and their |q|² in the device lane order.
int32_t batched_search(osk_view* v, int nq, int k, int UP, const uint64_t* const* d_accept,
                       uint64_t* d_shard_keys, int32_t* d_shard_counts, int64_t* d_visited, hipStream_t st) {
    int32_t rc = ensure_mfma(v, st);
    if (rc) return rc;
    const int S = v->n_shards, KS = v->mfma_KS;
    const int n_qb = (nq + 255) / 256;
    const int nq_pad = n_qb * 256;
    OSK_HIP(v->ws_qsplit.reserve((size_t)(nq_pad / 16) * KS * 2 * 1024));
    OSK_HIP(launch_split_rows(v->ws_q.as<float4>(), nq, UP, KS, nq_pad / 16, v->ws_qsplit.p, st));
    OSK_HIP(v->ws_cand_a.reserve(sizeof(uint64_t) * (size_t)nq * v->n_munits * 2 * kKC));
    MfmaParams mp{};
    mp.segs = v->d_segs.as<SegDev>();
    mp.units = v->d_munits.as<MfmaUnit>();
    mp.seg_split = v->d_seg_split.as<const void*>();
    mp.xsqrt = v->d_seg_xsqrt.as<const float*>();
    mp.accept = d_accept;
    mp.qsplit = v->ws_qsplit.p;
    mp.qnorm = v->ws_qnorm.as<float>();
    mp.cand = v->ws_cand_a.as<uint64_t>();
    mp.visited = reinterpret_cast<unsigned long long*>(d_visited);
    mp.n_units = v->n_munits;
    mp.KS = KS;
    mp.nq = nq;
    mp.nq_pad = std::min(nq_pad, (int)(v->ws_qnorm.cap / sizeof(float)));
    mp.sim = v->sim;
    mp.ablate = g_tuning.mfma_ablate;
    if (!v->d_mfma_full.p) {
        OSK_HIP(v->d_mfma_full.reserve(sizeof(unsigned long long)));
        OSK_HIP(hipMemsetAsync(v->d_mfma_full.p, 0, sizeof(unsigned long long), st));
    }
    mp.full_tiles = v->d_mfma_full.as<unsigned long long>();
    mp.n_shards = S;
    OSK_HIP(v->ws_akeys.reserve(sizeof(uint64_t) * (size_t)nq * S * kKC));
    OSK_HIP(v->ws_acounts.reserve(sizeof(int32_t) * (size_t)nq * S));
    if (!(g_tuning.mfma_ablate & 16)) {
        // pilot: the first tile of every unit, merged per (query, shard) → k'-th approx score =
        // a threshold no row below which can reach the shard's top-k'
        OSK_HIP(v->ws_pkeys.reserve(sizeof(uint64_t) * (size_t)nq * S * kKC));
        OSK_HIP(v->ws_pcounts.reserve(sizeof(int32_t) * (size_t)nq * S));
        MfmaParams pp = mp;
        pp.visited = nullptr;
        OSK_HIP(launch_mfma_cand(pp, n_qb, true, st));
        OSK_HIP(launch_merge_shards(v->ws_cand_a.as<uint64_t>(), v->n_munits * 2, v->d_shard_unit_begin.as<int32_t>(),
                                    S, nq, kKC, v->ws_pkeys.as<uint64_t>(), v->ws_pcounts.as<int32_t>(), st));
        mp.thr_keys = v->ws_pkeys.as<uint64_t>();
        mp.thr_counts = v->ws_pcounts.as<int32_t>();
    }
    OSK_HIP(launch_mfma_cand(mp, n_qb, false, st));
    rc = profile_end(v, st, true);
    if (rc) return rc;
    OSK_HIP(launch_merge_shards(v->ws_cand_a.as<uint64_t>(), v->n_munits * 2, v->d_shard_unit_begin.as<int32_t>(),
                                S, nq, kKC, v->ws_akeys.as<uint64_t>(), v->ws_acounts.as<int32_t>(), st));
    OSK_HIP(v->ws_flags.reserve(sizeof(int) * nq));
    OSK_HIP(hipMemsetAsync(v->ws_flags.p, 0, sizeof(int) * nq, st));
    RescoreParams rp{};
    rp.segs = v->d_segs.as<SegDev>();
    rp.seg_vrow_begin = v->d_seg_vrow.as<int64_t>();
    rp.akeys = v->ws_akeys.as<uint64_t>();
    rp.q = v->ws_q.p;
    rp.qnorm_dev = v->ws_qnorm.as<float>();
    rp.qnorm_approx = v->ws_qnorm.as<float>();
    rp.shard_maxnorm2 = v->d_shard_maxnorm2.as<float>();
    rp.shard_keys = d_shard_keys;
    rp.shard_counts = d_shard_counts;
    rp.flags = v->ws_flags.as<int>();
    rp.c = v->mfma_c;
    rp.n_shards = S;
    rp.n_segs = (int)v->segs.size();
    rp.units = v->units;
    rp.k = k;
    rp.sim = v->sim;
    OSK_HIP(launch_rescore(v->cfg, nq, rp, st));
    // certificate failures → exact streaming scan of those queries (rare; needs the flags on host)
    OSK_HIP(v->h_flags.reserve(sizeof(int) * nq));
    OSK_HIP(hipMemcpyAsync(v->h_flags.p, v->ws_flags.p, sizeof(int) * nq, hipMemcpyDeviceToHost, st));
    OSK_HIP(hipStreamSynchronize(st));
    const int* fl = static_cast<const int*>(v->h_flags.p);
    std::vector<int> fail;
    for (int q = 0; q < nq; ++q)
        if (fl[q]) fail.push_back(q);
    v->mfma_calls += 1;
    v->mfma_fallback_queries += (int64_t)fail.size();
    if (fail.empty() || g_tuning.mfma_ablate) return OSK_OK;
    const int nf = (int)fail.size();
    const int nf_pad = (nf + kMaxNQ - 1) / kMaxNQ * kMaxNQ;
    OSK_HIP(v->ws_fbq.reserve((size_t)nf_pad * UP * 16 + sizeof(float) * nf_pad));
    OSK_HIP(hipMemsetAsync(v->ws_fbq.p, 0, (size_t)nf_pad * UP * 16 + sizeof(float) * nf_pad, st));
    char* fbq = v->ws_fbq.as<char>();
    float* fbn = reinterpret_cast<float*>(fbq + (size_t)nf_pad * UP * 16);
    for (int i = 0; i < nf; ++i) {
        OSK_HIP(hipMemcpyAsync(fbq + (size_t)i * UP * 16, v->ws_q.as<char>() + (size_t)fail[i] * UP * 16,
                               (size_t)UP * 16, hipMemcpyDeviceToDevice, st));
        OSK_HIP(hipMemcpyAsync(fbn + i, v->ws_qnorm.as<float>() + fail[i], sizeof(float), hipMemcpyDeviceToDevice, st));
    }
    OSK_HIP(v->ws_fbkeys.reserve(sizeof(uint64_t) * (size_t)nf * S * k));
    OSK_HIP(v->ws_fbcounts.reserve(sizeof(int32_t) * (size_t)nf * S));
    const bool prof = v->profile;
    v->profile = false;
    rc = stream_search(v, fbq, fbn, nf, k, UP, d_accept, v->ws_fbkeys.as<uint64_t>(),
                       v->ws_fbcounts.as<int32_t>(), nullptr, st);
    v->profile = prof;
    if (rc) return rc;
    for (int i = 0; i < nf; ++i) {
        OSK_HIP(hipMemcpyAsync(d_shard_keys + (size_t)fail[i] * S * k, v->ws_fbkeys.as<uint64_t>() + (size_t)i * S * k,
                               sizeof(uint64_t) * S * k, hipMemcpyDeviceToDevice, st));
        OSK_HIP(hipMemcpyAsync(d_shard_counts + (size_t)fail[i] * S, v->ws_fbcounts.as<int32_t>() + (size_t)i * S,
                               sizeof(int32_t) * S, hipMemcpyDeviceToDevice, st));
    }
    return OSK_OK;
}

// The segment's int8 copy + per-row bound terms for the certified prefilter.  Built once.
int32_t ensure_sq8_seg(osk_seg* s, hipStream_t st) {
    std::lock_guard<std::mutex> lk(s->mu);
    if (s->d_q8) return OSK_OK;
    const int u8 = (s->dim + 15) / 16;
    void* q8 = nullptr;
    hipError_t e = hipMalloc(&q8, (size_t)std::max<int64_t>(1, s->n_rows) * u8 * 16);
    if (e != hipSuccess) {
        set_error(std::string("hipMalloc of the int8 prefilter copy failed: ") + hipGetErrorString(e));
        return OSK_ERR_OOM;
    }
    float4* aux = nullptr;
    e = hipMalloc(&aux, (size_t)std::max<int64_t>(1, s->n_rows) * sizeof(float4));
    if (e != hipSuccess) {
        (void)hipFree(q8);
        set_error(std::string("hipMalloc of the prefilter bound terms failed: ") + hipGetErrorString(e));
        return OSK_ERR_OOM;
    }
    OSK_HIP(launch_sq8_quantize(static_cast<const float4*>(s->d_rows), s->n_rows, s->units, s->units, u8, q8, aux,
                                0, st));
    // the 6-bit tier of single queries, where the dim has one and the tier is on (a node
    // that sets tune sq6 = 0 before staging never holds the copy; calibration frees it per segment)
    void* q6 = nullptr;
    float4* aux6 = nullptr;
    if (sq6_supported(s->dim) && g_tuning.sq6.load(std::memory_order_relaxed)) {
        // (stream-ordered allocations: the calibration frees them with hipFreeAsync behind the events of the
        // launches that read them, no device-wide wait — fold_probe)
        const int64_t b6 = sq6_bytes(s->n_rows, s->dim), ba = std::max<int64_t>(1, s->n_rows) * 16;
        e = hipMallocAsync(&q6, (size_t)(b6 - ba), st);
        if (e == hipSuccess) e = hipMallocAsync(reinterpret_cast<void**>(&aux6), (size_t)ba, st);
        if (e != hipSuccess) {
            if (q6) (void)hipFreeAsync(q6, st);
            (void)hipStreamSynchronize(st);
            (void)hipFree(q8);
            (void)hipFree(aux);
            set_error(std::string("hipMalloc of the 6-bit prefilter tier failed: ") + hipGetErrorString(e));
            return OSK_ERR_OOM;
        }
        OSK_HIP(launch_sq6_quantize(static_cast<const float4*>(s->d_rows), s->n_rows, s->units, s->dim, q6, aux6, st));
    }
    OSK_HIP(hipStreamSynchronize(st));
    s->d_q8 = q8;
    s->d_q8aux = aux;
    s->d_q6 = q6;
    s->d_q6aux = aux6;
    s->units8 = u8;
    return OSK_OK;
}

// The segment's int8 copy in sq8_mfma's tiled layout: blocks of 16 rows, per 64-dim k-step one
// contiguous 1 KiB slab (chunk-major: 16-dim chunk c of row r at c·256 + r·16 B), so each of the scan's
// load instructions reads 1 KiB contiguous and a 32-dim tail is the slab's first 512 B.  Built once, from
// the row-major int8 copy.
int32_t ensure_sq8t_seg(osk_seg* s, hipStream_t st, bool wide) {
    std::lock_guard<std::mutex> lk(s->mu);
    const int u8 = (s->dim + 15) / 16;
    const int64_t blocks = std::max<int64_t>(1, (s->n_rows + 15) / 16);
    if (!s->d_q8t) {
        const int ks = sq8_mfma_ks(u8);
        void* q8t = nullptr;
        hipError_t e = hipMalloc(&q8t, (size_t)blocks * ks * 1024);
        if (e != hipSuccess) {
            set_error(std::string("hipMalloc of the tiled int8 copy failed: ") + hipGetErrorString(e));
            return OSK_ERR_OOM;
        }
        OSK_HIP(launch_sq8_tile(s->d_q8, s->n_rows, u8, ks, q8t, st));
        OSK_HIP(hipStreamSynchronize(st));
        s->d_q8t = q8t;
    }
    // the wide kernel's own copy (osk_sq8w.hip launch_sq8w_build): codes with one scale per 16-row group,
    // tiled, and their bound terms per group (352 B per 16 rows).  Built the first time the cost model sends a
    // batch of this segment's view to the wide kernel (a node whose batches never take it does not
    // hold a second int8 copy — at 768 dims +768 B per row)
    if (wide && !s->d_q8w && sq8_wide_supported(u8)) {
        void* q8w = nullptr;
        float4* auxt = nullptr;
        hipError_t e = hipMalloc(&q8w, (size_t)blocks * sq8_wide_ks(u8) * 1024);
        if (e == hipSuccess) e = hipMalloc(&auxt, (size_t)blocks * kAuxGroupF4 * sizeof(float4));
        if (e != hipSuccess) {
            if (q8w) (void)hipFree(q8w);
            set_error(std::string("hipMalloc of the wide prefilter copy failed: ") + hipGetErrorString(e));
            return OSK_ERR_OOM;
        }
        OSK_HIP(launch_sq8w_build(static_cast<const float4*>(s->d_rows), s->n_rows, s->units, u8,
                                  s->sim == SIM_COSINE ? s->d_xnorm_f : nullptr, s->sim == SIM_COSINE ? 1 : 0, q8w, auxt,
                                  st));
        OSK_HIP(hipStreamSynchronize(st));
        s->d_q8w = q8w;
        s->d_q8auxt = auxt;
    }
    return OSK_OK;
}

int32_t ensure_sq8t(osk_view* v, hipStream_t st) {
    if (v->sq8t_ready) return OSK_OK;
    const int ns = (int)v->segs.size();
    std::vector<const void*> rows(ns);
    for (int i = 0; i < ns; ++i) {
        int32_t rc = ensure_sq8t_seg(v->segs[i], st, false);
        if (rc) return rc;
        rows[i] = v->segs[i]->d_q8t;
    }
    OSK_HIP(v->d_sq8_rows_t.reserve(sizeof(void*) * ns));
    OSK_HIP(hipMemcpyAsync(v->d_sq8_rows_t.p, rows.data(), sizeof(void*) * ns, hipMemcpyHostToDevice, st));
    OSK_HIP(hipStreamSynchronize(st));
    v->sq8t_ready = true;
    return OSK_OK;
}

// The wide kernel's inputs for a view (first batch the cost model sends to it): every segment's group-scaled
// copy and tiled bound terms, and the view's own tile table of quarters.
int32_t ensure_sq8w(osk_view* v, hipStream_t st) {
    if (v->sq8w_ready) return OSK_OK;
    int32_t rc = ensure_sq8t(v, st);
    if (rc) return rc;
    const int ns = (int)v->segs.size();
    std::vector<const void*> rows_w(ns), auxt(ns);
    for (int i = 0; i < ns; ++i) {
        rc = ensure_sq8t_seg(v->segs[i], st, true);
        if (rc) return rc;
        rows_w[i] = v->segs[i]->d_q8w;
        auxt[i] = v->segs[i]->d_q8auxt;
    }
    OSK_HIP(v->d_sq8_rows_w.reserve(sizeof(void*) * ns));
    OSK_HIP(v->d_sq8_auxt.reserve(sizeof(void*) * ns));
    OSK_HIP(hipMemcpyAsync(v->d_sq8_rows_w.p, rows_w.data(), sizeof(void*) * ns, hipMemcpyHostToDevice, st));
    OSK_HIP(hipMemcpyAsync(v->d_sq8_auxt.p, auxt.data(), sizeof(void*) * ns, hipMemcpyHostToDevice, st));
    if (sq8_wide_supported((v->segs.empty() ? 0 : v->segs[0]->units8)) && v->n_tiles > 0) {
        // The wide kernel's own tiles: its lists are per (tile, quarter) and every quarter's lists are
        // written for all 256 queries, so quarters of the scan tiles (≈ 244 rows at C2) would make the list
        // traffic rival the corpus.  Quarters here hold ≈ R / (2·CUs) rows, 256 … 16,384 (C2 ≈ 2k, C4 16k;
        // two to a few dozen per persistent workgroup), tiles never span segments, cut at multiples of 16.
        if (v->n_cus <= 0 &&
            (hipDeviceGetAttribute(&v->n_cus, hipDeviceAttributeMultiprocessorCount, v->device) != hipSuccess ||
             v->n_cus <= 0))
            v->n_cus = 256;
        double R = 0.0;
        for (const osk_seg* sg : v->segs) R += (double)sg->n_rows;
        // (≥ 512 dims: quarters of R / (8·CUs), so the first pass — one round of the persistent grid — covers
        // 1/8 of the rows, not 1/2, and the second pass's floors come early; list traffic is small beside
        // rows of ≥ 512 B)
        const int u8w = v->segs.empty() ? 1 : v->segs[0]->units8;
        const int qdiv = sq8_wide_ks(u8w) >= 8 ? 8 : 2;
        // (≤ 16,384 rows, round 5's best for the ring kernel; the rows kernel ran C4 b1024 in 16.05 ms at 32,768
        // against 16.42 (profiles/r06/tune14.jsonl) but a first-pass quarter that long can fill a queue: one C4
        // query in 256 took an exact re-scan, profiles/r06/rows_clocks_c4_b256_q32768.log)
        const int64_t qmax = 16384;
        const int64_t qr = g_tuning.sq8_wide_quarter_rows > 0
                               ? std::max<int64_t>(16, (int64_t)g_tuning.sq8_wide_quarter_rows & ~15ll)
                               : std::min<int64_t>(qmax, std::max<int64_t>(256, (int64_t)(R / ((double)qdiv * v->n_cus)) + 15 & ~15ll));
        const int64_t trows = 4 * qr;
        std::vector<TileDev> wt;
        v->wshard_tile_begin.assign(v->n_shards + 1, 0);
        for (int sh = 0; sh < v->n_shards; ++sh) {
            v->wshard_tile_begin[sh] = (int32_t)wt.size();
            for (int i = 0; i < ns; ++i) {
                if ((v->seg_shard.empty() ? 0 : v->seg_shard[i]) != sh) continue;
                const int64_t n = v->segs[i]->n_rows;
                if (n == 0) continue;
                const int64_t nt = (n + trows - 1) / trows;
                auto cut = [&](int64_t t) { return t >= nt ? n : (n * t / nt) & ~(int64_t)15; };
                for (int64_t t = 0; t < nt; ++t)
                    if (cut(t + 1) > cut(t)) wt.push_back(TileDev{i, sh, cut(t), cut(t + 1)});
            }
        }
        v->wshard_tile_begin[v->n_shards] = (int32_t)wt.size();
        v->n_wtiles = (int)wt.size();
        std::vector<int32_t> order(std::max<size_t>(1, wt.size()), 0), sqb(v->n_shards + 1);
        {   // interleaved over shards (as the scan tiles' order)
            std::vector<std::pair<double, int>> key;
            for (int sh = 0; sh < v->n_shards; ++sh) {
                const int t0 = v->wshard_tile_begin[sh], n = v->wshard_tile_begin[sh + 1] - t0;
                for (int j = 0; j < n; ++j) key.push_back({(j + 0.5) / n, t0 + j});
            }
            std::stable_sort(key.begin(), key.end(), [](auto& a, auto& b) { return a.first < b.first; });
            for (size_t i = 0; i < key.size(); ++i) order[i] = key[i].second;
        }
        for (int i = 0; i <= v->n_shards; ++i) sqb[i] = 4 * v->wshard_tile_begin[i];
        OSK_HIP(v->d_wtiles.reserve(sizeof(TileDev) * std::max<size_t>(1, wt.size())));
        OSK_HIP(v->d_wtile_order.reserve(sizeof(int32_t) * order.size()));
        OSK_HIP(v->d_wshard_tile_begin.reserve(sizeof(int32_t) * (v->n_shards + 1)));
        OSK_HIP(v->d_shard_quarter_begin.reserve(sizeof(int32_t) * sqb.size()));
        if (!wt.empty())
            OSK_HIP(hipMemcpyAsync(v->d_wtiles.p, wt.data(), sizeof(TileDev) * wt.size(), hipMemcpyHostToDevice, st));
        OSK_HIP(hipMemcpyAsync(v->d_wtile_order.p, order.data(), sizeof(int32_t) * order.size(), hipMemcpyHostToDevice, st));
        OSK_HIP(hipMemcpyAsync(v->d_wshard_tile_begin.p, v->wshard_tile_begin.data(), sizeof(int32_t) * (v->n_shards + 1),
                               hipMemcpyHostToDevice, st));
        OSK_HIP(hipMemcpyAsync(v->d_shard_quarter_begin.p, sqb.data(), sizeof(int32_t) * sqb.size(), hipMemcpyHostToDevice,
                               st));
        OSK_HIP(v->d_quarter_bm.reserve(sizeof(float4) * 4 * std::max<size_t>(1, wt.size())));
        OSK_HIP(launch_wide_quarter_max(v->d_wtiles.as<TileDev>(), v->n_wtiles, v->d_sq8_auxt.as<const float4*>(),
                                        v->d_quarter_bm.as<float4>(), st));
        // the quarters' descriptors, read by every workgroup's setup instead of recomputed (64 B each)
        OSK_HIP(v->d_wqtable.reserve((size_t)64 * 4 * std::max<size_t>(1, wt.size())));
        OSK_HIP(launch_wide_quarter_table(v->d_wtiles.as<TileDev>(), v->d_wtile_order.as<int32_t>(), 4 * v->n_wtiles,
                                          sq8_wide_ks(u8w), v->d_sq8_rows_w.p, v->d_sq8_auxt.p,
                                          v->d_seg_vrow.as<int64_t>(), v->d_quarter_bm.as<const float4>(),
                                          v->d_wqtable.p, st));
    }
    OSK_HIP(hipStreamSynchronize(st));
    v->sq8w_ready = true;
    return OSK_OK;
}

// Settle slices over the wave lists of a tile table (list = tile·4 + wave): kSliceLists lists each,
// never spanning shards (an empty shard gets one empty slice so its result is still written); each
// slice carries its L group (aligned chunks of kLGroupLists lists of the shard).
void settle_slices(const std::vector<int32_t>& shard_tile_begin, std::vector<int4>& sl, std::vector<int32_t>& ssb) {
    const int S = (int)shard_tile_begin.size() - 1;
    sl.clear();
    ssb.assign(S + 1, 0);
    for (int sh = 0; sh < S; ++sh) {
        ssb[sh] = (int32_t)sl.size();
        const int l0 = 4 * shard_tile_begin[sh], l1 = 4 * shard_tile_begin[sh + 1];
        if (l0 == l1) sl.push_back(make_int4(l0, l0, l0, l0));
        for (int l = l0; l < l1; l += kSliceLists) {
            const int ga = l0 + (l - l0) / kLGroupLists * kLGroupLists;
            sl.push_back(make_int4(l, std::min(l + kSliceLists, l1), ga, std::min(ga + kLGroupLists, l1)));
        }
    }
    ssb[S] = (int32_t)sl.size();
}

// Gather tiles for filtered scans over the compacted accepted ordinals (osk_filter.hip): one round of
// the chip's resident scan workgroups (CUs × 4) split over the segments by rows, at least one per
// non-empty segment, ordered by shard like the row tiles (so lists never span shards); gather tile
// j of nj of a segment covers ordinals [cnt·j/nj, cnt·(j+1)/nj) of its cnt accepted ones.  Built once.
int32_t ensure_gather(osk_view* v, hipStream_t st) {
    if (v->gather_ready) return OSK_OK;
    const int ns = (int)v->segs.size();
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, v->device) != hipSuccess || cus <= 0)
        cus = 256;
    const int64_t target = std::min<int64_t>((int64_t)cus * 4, std::max(1, v->n_tiles));
    int64_t total = 0;
    for (osk_seg* sg : v->segs) total += sg->n_rows;
    std::vector<int4> gt;
    std::vector<int32_t> gsb(v->n_shards + 1, 0);
    for (int sh = 0; sh < v->n_shards; ++sh) {
        gsb[sh] = (int32_t)gt.size();
        for (int i = 0; i < ns; ++i) {
            if (v->seg_shard[i] != sh || v->segs[i]->n_rows == 0) continue;
            const int64_t nj = std::max<int64_t>(1, (int64_t)((double)v->segs[i]->n_rows * target / std::max<int64_t>(1, total)));
            for (int64_t j = 0; j < nj; ++j) gt.push_back(make_int4(i, sh, (int)j, (int)nj));
        }
    }
    gsb[v->n_shards] = (int32_t)gt.size();
    std::vector<int4> sl;
    std::vector<int32_t> ssb;
    settle_slices(gsb, sl, ssb);
    // each segment's tile range in the row-tile table (tiles of a segment are contiguous)
    std::vector<TileDev> tiles(v->n_tiles);
    if (v->n_tiles)
        OSK_HIP(hipMemcpyAsync(tiles.data(), v->d_tiles.p, sizeof(TileDev) * v->n_tiles, hipMemcpyDeviceToHost, st));
    OSK_HIP(hipStreamSynchronize(st));
    std::vector<int2> seg_tiles(ns, make_int2(0, 0));
    for (int t = 0; t < v->n_tiles; ++t) {
        int2& r = seg_tiles[tiles[t].seg];
        if (r.x == r.y) r = make_int2(t, t + 1);
        else r.y = t + 1;
    }
    v->n_gtiles = (int)gt.size();
    v->n_gslices = (int)sl.size();
    OSK_HIP(v->d_gtiles.reserve(sizeof(int4) * std::max<size_t>(1, gt.size())));
    OSK_HIP(v->d_gslices.reserve(sizeof(int4) * sl.size()));
    OSK_HIP(v->d_gshard_slice_begin.reserve(sizeof(int32_t) * ssb.size()));
    OSK_HIP(v->d_seg_tiles.reserve(sizeof(int2) * ns));
    OSK_HIP(v->ws_tcnt.reserve(sizeof(int32_t) * std::max(1, v->n_tiles)));
    OSK_HIP(v->ws_scnt.reserve(sizeof(int32_t) * ns));
    OSK_HIP(v->ws_comp.reserve(sizeof(uint32_t) * std::max<int64_t>(1, total)));
    if (!gt.empty())
        OSK_HIP(hipMemcpyAsync(v->d_gtiles.p, gt.data(), sizeof(int4) * gt.size(), hipMemcpyHostToDevice, st));
    OSK_HIP(hipMemcpyAsync(v->d_gslices.p, sl.data(), sizeof(int4) * sl.size(), hipMemcpyHostToDevice, st));
    OSK_HIP(hipMemcpyAsync(v->d_gshard_slice_begin.p, ssb.data(), sizeof(int32_t) * ssb.size(), hipMemcpyHostToDevice, st));
    OSK_HIP(hipMemcpyAsync(v->d_seg_tiles.p, seg_tiles.data(), sizeof(int2) * ns, hipMemcpyHostToDevice, st));
    OSK_HIP(hipStreamSynchronize(st));
    v->gather_ready = true;
    return OSK_OK;
}

int32_t ensure_sq8(osk_view* v, hipStream_t st) {
    if (v->sq8_ready) return OSK_OK;
    const int ns = (int)v->segs.size();
    std::vector<const void*> rows(ns);
    std::vector<const float4*> aux(ns);
    for (int i = 0; i < ns; ++i) {
        int32_t rc = ensure_sq8_seg(v->segs[i], st);
        if (rc) return rc;
        rows[i] = v->segs[i]->d_q8;
        aux[i] = v->segs[i]->d_q8aux;
    }
    v->units8 = (v->dim + 15) / 16;
    {
        std::vector<int4> sl;
        std::vector<int32_t> ssb;
        settle_slices(v->shard_tile_begin, sl, ssb);
        v->n_slices = (int)sl.size();
        OSK_HIP(v->d_slices.reserve(sizeof(int4) * sl.size()));
        OSK_HIP(v->d_shard_slice_begin.reserve(sizeof(int32_t) * ssb.size()));
        OSK_HIP(hipMemcpyAsync(v->d_slices.p, sl.data(), sizeof(int4) * sl.size(), hipMemcpyHostToDevice, st));
        OSK_HIP(hipMemcpyAsync(v->d_shard_slice_begin.p, ssb.data(), sizeof(int32_t) * ssb.size(),
                               hipMemcpyHostToDevice, st));
    }
    // rounding bounds of the fp32 device order over n = 4·units products: γ_n ≤ n·2^-24
    // (any summation tree); gam = γ_n/2 with a 2× margin, g2 ≥ γ_{n+2} with margin.
    const double n = 4.0 * v->units;
    v->sq8_gam = (float)((n + 8.0) * std::ldexp(1.0, -24));
    v->sq8_g2 = (float)((n + 8.0) * std::ldexp(1.0, -23));
    v->sq8_cos_slack = (float)((n + 8.0) * std::ldexp(1.0, -23) + std::ldexp(1.0, -18));
    OSK_HIP(v->d_sq8_rows.reserve(sizeof(void*) * ns));
    OSK_HIP(v->d_sq8_aux.reserve(sizeof(void*) * ns));
    OSK_HIP(hipMemcpyAsync(v->d_sq8_rows.p, rows.data(), sizeof(void*) * ns, hipMemcpyHostToDevice, st));
    OSK_HIP(hipMemcpyAsync(v->d_sq8_aux.p, aux.data(), sizeof(void*) * ns, hipMemcpyHostToDevice, st));
    // the 6-bit tier: used only when every segment has one
    std::vector<const void*> rows6(ns);
    std::vector<const float4*> aux6(ns);
    bool all6 = ns > 0;
    for (int i = 0; i < ns; ++i) {
        rows6[i] = v->segs[i]->d_q6;
        aux6[i] = v->segs[i]->d_q6aux;
        all6 = all6 && rows6[i] && aux6[i];
    }
    if (all6) {
        OSK_HIP(v->d_sq6_rows.reserve(sizeof(void*) * ns));
        OSK_HIP(v->d_sq6_aux.reserve(sizeof(void*) * ns));
        OSK_HIP(hipMemcpyAsync(v->d_sq6_rows.p, rows6.data(), sizeof(void*) * ns, hipMemcpyHostToDevice, st));
        OSK_HIP(hipMemcpyAsync(v->d_sq6_aux.p, aux6.data(), sizeof(void*) * ns, hipMemcpyHostToDevice, st));
    }
    OSK_HIP(hipStreamSynchronize(st));
    v->sq6_ready = all6;
    v->sq8_ready = true;
    return OSK_OK;
}

// The 6-bit tier's calibration, folded without waiting: when this view's last probe has
// landed (its event completed), its per-segment int8 re-bound counts join the segments' calibration; a
// segment with kSq6Probes probes keeps the tier, or turns it off (re-bounds above sq6_probe_pct % of the
// rows probed) and frees its 6-bit copy — stream-ordered, with no host or device-wide wait:
//  * only a probing segment (state 0) can turn off, so only launches issued while some segment of the view
//    probes register an event (sq6_track_launch); a kept segment (state 1) never frees its copy early;
//  * a search holds the shared side of g_sq6_free_mu from its state check to that registration, so once the
//    freeing call holds the exclusive side (briefly: no waiting under it) every launch that may read the
//    copy is registered, and every later search sees state 2 and leaves the tier alone;
//  * the freeing call's stream waits on the events of the registered launches still in flight over the
//    segment (other views' streams included), then hipFreeAsync releases the copy on that stream.
std::shared_mutex g_sq6_free_mu;
struct Sq6Inflight {
    int device;
    hipEvent_t ev;
    std::vector<const osk_seg*> segs;
};
std::mutex g_sq6_inflight_mu;                       // (inner to g_sq6_free_mu)
std::vector<Sq6Inflight> g_sq6_inflight;            // launches over probing segments, not yet seen complete
std::vector<std::pair<int, hipEvent_t>> g_sq6_ev_pool;

// (g_sq6_inflight_mu held) drop the entries whose launches have completed; their events go back to the pool
void sq6_prune_locked() {
    size_t j = 0;
    for (size_t i = 0; i < g_sq6_inflight.size(); ++i) {
        if (hipEventQuery(g_sq6_inflight[i].ev) == hipSuccess)
            g_sq6_ev_pool.push_back({g_sq6_inflight[i].device, g_sq6_inflight[i].ev});
        else
            g_sq6_inflight[j++] = std::move(g_sq6_inflight[i]);
    }
    g_sq6_inflight.resize(j);
}

// A segment being destroyed leaves the in-flight records (its launches have completed: the destructor's hipFree
// calls synchronise the device), so a segment later allocated at the same address never waits on them.
void sq6_forget_segment(const osk_seg* sg) {
    std::lock_guard<std::mutex> lk(g_sq6_inflight_mu);
    for (Sq6Inflight& f : g_sq6_inflight) f.segs.erase(std::remove(f.segs.begin(), f.segs.end(), sg), f.segs.end());
    sq6_prune_locked();
}

// A 6-bit launch over a view with a probing segment: record its completion (caller holds the shared side
// of g_sq6_free_mu, and the view's device is current).
int32_t sq6_track_launch(const osk_view* v, hipStream_t st) {
    std::lock_guard<std::mutex> lk(g_sq6_inflight_mu);
    sq6_prune_locked();
    hipEvent_t ev = nullptr;
    for (size_t i = 0; i < g_sq6_ev_pool.size(); ++i)
        if (g_sq6_ev_pool[i].first == v->device) {
            ev = g_sq6_ev_pool[i].second;
            g_sq6_ev_pool.erase(g_sq6_ev_pool.begin() + (ptrdiff_t)i);
            break;
        }
    if (!ev) OSK_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    hipError_t e = hipEventRecord(ev, st);
    if (e != hipSuccess) {
        g_sq6_ev_pool.push_back({v->device, ev});
        OSK_HIP(e);
    }
    g_sq6_inflight.push_back(Sq6Inflight{v->device, ev, std::vector<const osk_seg*>(v->segs.begin(), v->segs.end())});
    return OSK_OK;
}

int32_t fold_probe(osk_view* v, hipStream_t st) {
    if (!v->probe_pending || hipEventQuery(v->ev_probe) != hipSuccess) return OSK_OK;
    v->probe_pending = false;
    const unsigned long long* rb = static_cast<const unsigned long long*>(v->h_seg_rebound.p);
    std::vector<osk_seg*> off;
    for (size_t i = 0; i < v->segs.size(); ++i) {
        osk_seg* sg = v->segs[i];
        std::lock_guard<std::mutex> lk(sg->mu);
        if (sg->sq6_state.load() != 0) continue;
        sg->sq6_probe_rows += sg->n_rows;
        sg->sq6_probe_rebound += (int64_t)rb[i];
        if (++sg->sq6_probes < kSq6Probes) continue;
        const bool keep = (double)sg->sq6_probe_rebound * 100.0 <=
                          (double)sg->sq6_probe_rows * (double)g_tuning.sq6_probe_pct;
        sg->sq6_state.store(keep ? 1 : 2, std::memory_order_release);
        if (!keep) off.push_back(sg);
    }
    if (off.empty()) return OSK_OK;
    std::unique_lock<std::shared_mutex> ex(g_sq6_free_mu);
    std::lock_guard<std::mutex> lk(g_sq6_inflight_mu);
    sq6_prune_locked();
    for (const Sq6Inflight& f : g_sq6_inflight) {
        bool reads = false;
        for (const osk_seg* sg : off) reads = reads || std::find(f.segs.begin(), f.segs.end(), sg) != f.segs.end();
        if (reads) OSK_HIP(hipStreamWaitEvent(st, f.ev, 0));
    }
    for (osk_seg* sg : off) {
        std::lock_guard<std::mutex> sl(sg->mu);
        if (sg->d_q6) OSK_HIP(hipFreeAsync(sg->d_q6, st));
        if (sg->d_q6aux) OSK_HIP(hipFreeAsync(sg->d_q6aux, st));
        sg->d_q6 = nullptr;
        sg->d_q6aux = nullptr;
    }
    return OSK_OK;
}

// The prefilter's two int8 MFMA kernels, in µs for this view's R rows (measured end to end on MI355X,
// DESIGN.md §3c): sq8_mfma per launch of ≤ 32 queries streams R·(int8 row + 16-B bound terms) at ≈ 4.3 TB/s
// + ≈ 165 µs + 0.28 µs per dim (pilot, merge, settle, re-score); the wide kernel per launch of ≤ 256 queries
// ≈ R·KS·0.031 ns (it is issue-bound, not HBM-bound: C4 6.35 ms per 256 at b1024, C3 4.07 ms at b256, round 5
// with deferred insertions, profiles/r05d/) + ≈ 300 µs (pilot, two passes, floors, settle: C2 0.33 ms per 256).
double sq8_narrow_us(double R, int nq, int u8, int dim) {
    return (double)((nq + 31) / 32) * (R * (16.0 * u8 + 16.0) / 4.3e6 + 165.0 + 0.28 * dim);
}
double sq8_wide_us(double R, int nq, int u8) {
    return (double)((nq + kWideQ - 1) / kWideQ) * (R * sq8_wide_ks(u8) * 0.031e-3 + 300.0);
}
// the wide kernel takes an unfiltered batch of ≥ sq8_wide_min queries of ≤ 768 dims when the model has it
// cheaper than sq8_mfma (C4: from about 96 queries)
bool sq8_wide_pick(const osk_view* v, int nq, bool filtered) {
    const int u8 = (v->dim + 15) / 16;
    if (filtered || !sq8_wide_supported(u8) || g_tuning.sq8_wide_min <= 0 || nq < g_tuning.sq8_wide_min ||
        g_tuning.sq8_mfma_min <= 0 || nq < g_tuning.sq8_mfma_min)
        return false;
    double R = 0.0;
    for (const osk_seg* sg : v->segs) R += (double)sg->n_rows;
    return g_tuning.sq8_wide_force || sq8_wide_us(R, nq, u8) <= sq8_narrow_us(R, nq, u8, v->dim);
}

// Certified int8 prefilter search (float32, k ≤ kKQ): int8 scan → settle per slice of tiles (exact
// re-score of the rows the certificate cannot exclude; a tile whose list overflowed is re-scanned
// exactly inside the settle) → per-shard merge.  Nothing waits on the host.
// ws_q / ws_qnorm hold the padded fp32 queries and |q|² (device order).
int32_t sq8_search(osk_view* v, const void* d_queries, int nq, int k, int UP, const uint64_t* const* d_accept,
                   uint64_t* d_shard_keys, int32_t* d_shard_counts, int64_t* d_visited, hipStream_t st) {
    int32_t rc = ensure_sq8(v, st);
    if (rc) return rc;
    const int u8 = v->units8, S = v->n_shards;
    const int nq_pad = (nq + kMaxNQ - 1) / kMaxNQ * kMaxNQ;
    // batches of ≥ sq8_mfma_min queries: the int8 MFMA scan, 16 queries per launch; else the VALU
    // scan, ≤ 8 per launch.  Filtered VALU scans run over the compacted accepted ordinals.  A single
    // unfiltered query scans the 6-bit tier where the view has one.
    const bool use_mfma = g_tuning.sq8_mfma_min > 0 && nq >= g_tuning.sq8_mfma_min && sq8_mfma_supported(u8);
    // large unfiltered batches of ≤ 768-dim rows: one corpus pass per kWideQ queries (osk_sq8w.hip)
    const bool use_wide = use_mfma && !g_tuning.sq8_force_fallback && sq8_wide_pick(v, nq, d_accept != nullptr);
    // the 6-bit tier: single unfiltered queries, every segment's calibration probing or on.  The shared
    // lock keeps a segment's copy alive from this check to the launches (fold_probe frees it under the
    // exclusive one, with hipFreeAsync behind the events of the launches still reading it: no device wait)
    rc = fold_probe(v, st);
    if (rc) return rc;
    std::shared_lock<std::shared_mutex> tier_lock(g_sq6_free_mu, std::defer_lock);
    bool use6 = nq == 1 && !d_accept && !use_mfma && v->sq6_ready && g_tuning.sq6;
    bool probing = false;
    if (use6) {
        tier_lock.lock();
        for (const osk_seg* sg : v->segs) {
            const int st6 = sg->sq6_state.load(std::memory_order_acquire);
            use6 = use6 && st6 != 2 && sg->d_q6;
            probing |= st6 == 0;
        }
    }
    // calibration: this call counts its int8 re-bounds per segment (one probe in flight per view)
    const bool probe6 = use6 && probing && !v->probe_pending;
    const int ns = (int)v->segs.size();
    if (probe6) {
        OSK_HIP(v->d_seg_rebound.reserve(sizeof(unsigned long long) * ns));
        OSK_HIP(v->h_seg_rebound.reserve(sizeof(unsigned long long) * ns));
        if (!v->ev_probe) OSK_HIP(hipEventCreateWithFlags(&v->ev_probe, hipEventDisableTiming));
        OSK_HIP(hipMemsetAsync(v->d_seg_rebound.p, 0, sizeof(unsigned long long) * ns, st));
    }
    OSK_HIP(v->ws_q8.reserve((size_t)nq_pad * u8 * 16));
    OSK_HIP(v->ws_qc.reserve(sizeof(float4) * nq_pad));
    OSK_HIP(v->ws_flags.reserve(sizeof(int) * nq));
    Sq6Prep q6{};
    if (use6) {
        q6.C = sq6_chunks(v->dim);
        q6.floor_n = S * (kFloorBuckets + 1) * kFloorStride;   // buckets + the floor cell per shard
        OSK_HIP(v->ws_q6.reserve((size_t)nq_pad * 256 * q6.C));
        OSK_HIP(v->ws_qc6.reserve(sizeof(float4) * nq_pad));
        OSK_HIP(v->ws_floor.reserve(sizeof(uint32_t) * (size_t)nq_pad * q6.floor_n));
        q6.q6 = v->ws_q6.as<uint32_t>();
        q6.qc6 = v->ws_qc6.as<float4>();
        q6.floor = v->ws_floor.as<uint32_t>();
    }
    // one launch: padded fp32 queries, |q|² (device order), int8 queries + bound terms (and the 6-bit
    // tier's query form, floor buckets zeroed), flags = 0
    OSK_HIP(launch_sq8_prep(v->cfg, static_cast<const float*>(d_queries), v->dim, nq, nq_pad, UP, u8,
                            v->ws_q.as<float4>(), v->ws_qnorm.as<float>(), v->ws_q8.p, v->ws_qc.as<float4>(),
                            v->ws_flags.as<int>(), st, q6));
    const bool gather = d_accept && !use_mfma && g_tuning.filter_gather;
    if (gather) {
        rc = ensure_gather(v, st);
        if (rc) return rc;
    }
    int n_scan_tiles = gather ? v->n_gtiles : v->n_tiles;
    if (use_wide) {   // its own copy and tile table (ensure_sq8w)
        rc = ensure_sq8w(v, st);
        if (rc) return rc;
        n_scan_tiles = v->n_wtiles;
    }
    const size_t nl = (size_t)nq * 4 * n_scan_tiles * kKQ;
    OSK_HIP(v->ws_sq8cand.reserve(sizeof(uint64_t) * nl));
    OSK_HIP(v->ws_sq8lb.reserve(sizeof(uint32_t) * nl));
    OSK_HIP(v->ws_lbmax.reserve(sizeof(uint32_t) * (size_t)nq * 4 * n_scan_tiles));
    Sq8Params p{};
    p.segs = v->d_segs.as<SegDev>();
    p.tiles = v->d_tiles.as<TileDev>();
    p.accept = d_accept;
    p.rows8 = v->d_sq8_rows.as<const int4*>();
    p.aux = v->d_sq8_aux.as<const float4*>();
    p.seg_vrow = v->d_seg_vrow.as<int64_t>();
    p.cand = v->ws_sq8cand.as<uint64_t>();
    p.cand_lb = v->ws_sq8lb.as<uint32_t>();
    p.list_lbmax = v->ws_lbmax.as<uint32_t>();
    p.visited = reinterpret_cast<unsigned long long*>(d_visited);
    p.n_tiles = n_scan_tiles;
    p.n_lists = 4 * n_scan_tiles;
    p.units8 = u8;
    p.sim = v->sim;
    p.gam = v->sq8_gam;
    p.g2 = v->sq8_g2;
    p.cos_slack = v->sq8_cos_slack;
    if (gather) {   // accepted ordinals of every segment, compacted (count, then prefix + write)
        FilterParams fp{};
        fp.segs = v->d_segs.as<SegDev>();
        fp.tiles = v->d_tiles.as<TileDev>();
        fp.accept = d_accept;
        fp.seg_vrow = v->d_seg_vrow.as<int64_t>();
        fp.seg_tiles = v->d_seg_tiles.as<int2>();
        fp.tcnt = v->ws_tcnt.as<int32_t>();
        fp.scnt = v->ws_scnt.as<int32_t>();
        fp.comp = v->ws_comp.as<uint32_t>();
        fp.n_tiles = v->n_tiles;
        fp.n_segs = (int)v->segs.size();
        OSK_HIP(launch_filter_compact(fp, st));
        p.gtiles = v->d_gtiles.as<int4>();
        p.comp = fp.comp;
        p.scnt = fp.scnt;
        p.gather_min = g_tuning.gather_min;
    }
    const int chunk = use_wide ? kWideQ : use_mfma ? (int)g_tuning.sq8_mfma_queries : kMaxNQ;
    if (use_mfma) {
        rc = ensure_sq8t(v, st);
        if (rc) return rc;
        p.rows8t = v->d_sq8_rows_t.as<const int4*>();
        p.auxt = v->d_sq8_auxt.as<const float4*>();
        const size_t qmax = use_wide ? kWideQ : kMfmaQueries;
        // pilot keys: per (query, list) of the table the launch walks — the wide kernel's own quarters
        // (4 per wide tile, qi·4·n_wtiles + list) or the scan tiles' (64 sampled keys per tile); the two
        // tables differ in size (tiles_target, views past ≈ 400M rows), so size by the one in use
        const size_t pilot_keys = use_wide ? qmax * 4 * (size_t)std::max(1, v->n_wtiles)
                                           : qmax * 64 * (size_t)std::max(1, v->n_tiles);
        OSK_HIP(v->ws_pilot.reserve(sizeof(uint64_t) * pilot_keys));
        OSK_HIP(v->ws_thr.reserve(sizeof(uint64_t) * qmax * S * 64));
        OSK_HIP(v->ws_thr_counts.reserve(sizeof(int32_t) * qmax * S));
        if (use_wide) OSK_HIP(v->ws_wfloor.reserve(sizeof(uint32_t) * 2 * kWideQ * S));
    }
    for (int q0 = 0; q0 < nq; q0 += chunk) {
        p.q0 = q0;
        p.q_count = std::min(chunk, nq - q0);
        p.q8 = v->ws_q8.as<int4>() + (size_t)q0 * u8;
        p.qc = v->ws_qc.as<float4>() + q0;
        p.qn_dev = v->ws_qnorm.as<float>() + q0;
        hipEvent_t e0 = v->profile && q0 == 0 ? v->ev0 : nullptr;
        hipEvent_t e1 = v->profile && q0 + chunk >= nq ? v->ev1 : nullptr;
        if (use_wide) {
            // pilot: the first step of every quarter → per (query, quarter) the best lower-bound key (and the
            // quarter's list maximum zeroed) → per (query, shard) the k-th best of them floors the main pass
            if (v->n_cus <= 0 &&
                (hipDeviceGetAttribute(&v->n_cus, hipDeviceAttributeMultiprocessorCount, v->device) != hipSuccess ||
                 v->n_cus <= 0))
                v->n_cus = 256;
            // persistent workgroups: one per CU (sq8_wide_grid overrides it: the tests' LDS-cap grid doubling)
            const int wgrid = g_tuning.sq8_wide_grid > 0 ? (int)g_tuning.sq8_wide_grid : v->n_cus;
            p.wide_grid = wgrid;
            p.rows8t = v->d_sq8_rows_w.as<const int4*>();   // (the wide copy: one scale per 16-row group)
            p.tiles = v->d_wtiles.as<TileDev>();
            p.tile_order = v->d_wtile_order.as<int32_t>();
            p.k = k;
            p.n_shards = S;
            p.ablate = g_tuning.sq8_mfma_ablate;
            p.counters = v->d_counters.as<unsigned long long>();   // (testing build: event counts)
            p.pilot = 1;
            // (0: 128 rows per quarter, 256 at ≥ 512 dims, where the pilot's steps are 32 rows and the better
            // floors pay: C3 b256 3.76 → 3.71 ms, C4's 96 dims 22.98 → 23.27 ms, profiles/r05p/tune50_*)
            // At least ≈ 64k pilot rows per shard: the floor is the k-th best of the shard's quarter maxima, so a
            // shard of few quarters (6.5M rows over 8 shards: 64 quarters of 12.7k rows) sampled at 128 rows a
            // quarter floored the first pass at ≈ its 1,000th best row, and the rows kernel's queues overflowed for
            // every query (exact re-scans of the overflowed quarters); up to 1,024 rows a quarter.
            const int prows = g_tuning.sq8_wide_pilot_rows.load();
            int pr = prows > 0 ? prows : (sq8_wide_ks(u8) >= 8 ? 256 : kWidePilotRowsDefault);
            if (prows <= 0) {
                const int qps = std::max(1, 4 * v->n_wtiles / std::max(1, S));   // quarters per shard
                const int want = (kWidePilotSample + qps - 1) / qps;
                pr = std::max(pr, std::min(1024, (want + 127) / 128 * 128));
            }
            p.pilot_rows = pr;
            p.wide_defer = g_tuning.sq8_wide_defer;
            p.pilot_keys = v->ws_pilot.as<uint64_t>();
            p.quarter_begin = 0;
            p.quarter_end = 0;
            p.floors = nullptr;
            p.quarter_bm = v->d_quarter_bm.as<const float4>();
            p.wide_qtable = v->d_wqtable.p;
            p.wide_claim = g_tuning.sq8_wide_rows_claim;
            // ≤ 128 dims: the pilot and the main passes without a step barrier (sq8_wide_rows, osk_sq8w.hip)
            const bool rows = g_tuning.sq8_wide_rows && sq8_wide_rows_supported(u8);
            p.wide_qcap = rows ? (int)g_tuning.sq8_wide_rows_qcap : 0;
            if (rows)
                OSK_HIP(launch_sq8_wide_rows(p, st, e0, nullptr));
            else
                OSK_HIP(launch_sq8_wide(p, st, e0, nullptr));
            const int nql = 4 * v->n_wtiles;
            const int32_t* sqb = v->d_shard_quarter_begin.as<int32_t>();
            uint32_t* floor_a = v->ws_wfloor.as<uint32_t>();
            uint32_t* floor_b = floor_a + (size_t)kWideQ * S;
            OSK_HIP(launch_wide_floor(nullptr, v->ws_pilot.as<uint64_t>(), nql, sqb, S, p.q_count, k, nullptr, floor_a,
                                      st));
            p.pilot = 0;
            p.floors = floor_a;
            // two passes: the first 1/phase of the quarters (tile order: every shard) under the pilot's floors,
            // then the rest under floors raised by the first pass's list maxima (the lists of the second pass
            // read as empty until it writes them)
            const int phase = g_tuning.sq8_wide_phase;
            // (the first pass takes whole rounds of the persistent grid, at least one: a small view's 1/phase
            // would idle the chip, and a partial round leaves a tail)
            const int rounds = std::max(1, (int)std::lround((double)nql / ((double)phase * wgrid)));
            const int n_a = phase > 1 ? std::min(nql / 2, rounds * wgrid) : 0;
            auto main_pass = [&](hipEvent_t ev) {
                return rows ? launch_sq8_wide_rows(p, st, nullptr, ev) : launch_sq8_wide(p, st, nullptr, ev);
            };
            if (n_a > 0) {   // (the pilot zeroed every list maximum: the second pass's read as empty)
                uint32_t* lbm = p.list_lbmax + (size_t)q0 * nql;
                p.quarter_end = n_a;
                OSK_HIP(main_pass(nullptr));
                OSK_HIP(launch_wide_floor(lbm, nullptr, nql, sqb, S, p.q_count, k, floor_a, floor_b, st));
                p.quarter_begin = n_a;
                p.quarter_end = 0;
                p.floors = floor_b;
            }
            OSK_HIP(main_pass(e1));
        } else if (use_mfma) {
            // pilot: 16 sampled rows per wave → per (query, tile) the top k sampled lower bounds →
            // per (query, shard) the top k; its k-th floors the main pass's quick thresholds
            // (sq8_mfma comment)
            p.k = k;
            p.n_shards = S;
            p.nt = g_tuning.sq8_mfma_nt;
            p.ring_slots = sq8_ring_slots(u8, p.q_count > 16 ? 2 : 1, g_tuning.sq8_mfma_ring);
            p.ablate = g_tuning.sq8_mfma_ablate;
            p.pilot = 1;
            p.pilot_keys = v->ws_pilot.as<uint64_t>();
            OSK_HIP(launch_sq8_mfma(p, st, e0, nullptr));
            OSK_HIP(launch_merge_shards(v->ws_pilot.as<uint64_t>(), v->n_tiles, v->d_shard_tile_begin.as<int32_t>(),
                                        S, p.q_count, k, v->ws_thr.as<uint64_t>(), v->ws_thr_counts.as<int32_t>(), st));
            p.pilot = 0;
            p.thr_keys = v->ws_thr.as<uint64_t>();
            p.thr_counts = v->ws_thr_counts.as<int32_t>();
            OSK_HIP(launch_sq8_mfma(p, st, nullptr, e1));
        } else if (use6) {
            p.rows6 = v->d_sq6_rows.as<const void*>();
            p.aux6 = v->d_sq6_aux.as<const float4*>();
            p.q6 = v->ws_q6.as<int4>() + (size_t)q0 * 16 * q6.C;
            p.qc6 = v->ws_qc6.as<float4>() + q0;
            p.floor = q6.floor;
            p.k = k;
            p.n_shards = S;
            p.counters = v->d_counters.as<unsigned long long>();
            p.ablate = g_tuning.sq8_mfma_ablate;
            p.tile_order = v->d_tile_order.as<int32_t>();
            if (v->n_cus <= 0 &&
                (hipDeviceGetAttribute(&v->n_cus, hipDeviceAttributeMultiprocessorCount, v->device) != hipSuccess ||
                 v->n_cus <= 0))
                v->n_cus = 256;
            p.wide_grid = v->n_cus;   // (the persistent re-bound's grid: 4 workgroups per CU)
            p.n_segs = ns;
            p.rb_stride = g_tuning.sq6_rebound_stride;
            p.rb_retest = g_tuning.sq6_rebound_retest;
            p.rb_wg_per_cu = g_tuning.sq6_rebound_wgs;
            OSK_HIP(v->ws_cand6.reserve(sizeof(uint2) * (size_t)p.n_lists * kSq6Cap));
            OSK_HIP(v->ws_cnt6.reserve(sizeof(int32_t) * (size_t)nq * p.n_lists));
            p.cand6 = v->ws_cand6.as<uint2>();
            p.cnt6 = v->ws_cnt6.as<int32_t>();
            p.cap6 = kSq6Cap;
            p.seg_rebound = probe6 ? v->d_seg_rebound.as<unsigned long long>() : nullptr;
            OSK_HIP(launch_sq6_scan(p, v->dim, st, e0, e1));
            if (probing) {   // a segment may still turn the tier off: its free waits for this launch
                rc = sq6_track_launch(v, st);
                if (rc) return rc;
            }
        } else {
            OSK_HIP(launch_sq8_scan(p.q_count, p, st, e0, e1));
        }
    }
    rc = profile_end(v, st, false);
    if (rc) return rc;
    const int n_slices = gather ? v->n_gslices : v->n_slices;
    OSK_HIP(v->ws_part.reserve(sizeof(uint64_t) * (size_t)nq * n_slices * k));
    SettleParams sp{};
    sp.slices = gather ? v->d_gslices.as<int4>() : v->d_slices.as<int4>();
    sp.shard_slice_begin = gather ? v->d_gshard_slice_begin.as<int32_t>() : v->d_shard_slice_begin.as<int32_t>();
    sp.tiles = v->d_tiles.as<TileDev>();
    sp.gtiles = p.gtiles;
    sp.comp = p.comp;
    sp.scnt = p.scnt;
    sp.gather_min = p.gather_min;   // the scan's split, exactly
    sp.accept = d_accept;
    sp.part = v->ws_part.as<uint64_t>();
    sp.n_slices = n_slices;
    sp.segs = v->d_segs.as<SegDev>();
    sp.seg_vrow = v->d_seg_vrow.as<int64_t>();
    sp.cand = p.cand;
    sp.cand_lb = p.cand_lb;
    sp.list_lbmax = p.list_lbmax;
    sp.q = v->ws_q.p;
    sp.qnorm = v->ws_qnorm.as<float>();
    sp.shard_keys = d_shard_keys;
    sp.shard_counts = d_shard_counts;
    sp.flags = v->ws_flags.as<int>();
    sp.counters = v->d_counters.as<unsigned long long>();
    sp.n_lists = 4 * n_scan_tiles;
    sp.scan_R = use_mfma ? kMfmaScanR : use6 ? kSq6ScanR : 64 / sq8_lanes(u8);
    sp.n_shards = S;
    sp.n_segs = (int)v->segs.size();
    sp.units = v->units;
    sp.k = k;
    sp.sim = v->sim;
    sp.force_fail = g_tuning.sq8_force_fallback;
    if (g_tuning.settle_trace) {
        OSK_HIP(v->ws_trace.reserve(sizeof(unsigned long long) * 8 * (size_t)nq * n_slices));
        sp.trace = v->ws_trace.as<unsigned long long>();
    }
    if (use_wide) {
        sp.tiles = v->d_wtiles.as<TileDev>();
        sp.shard_tile_begin = v->d_wshard_tile_begin.as<int32_t>();
        OSK_HIP(launch_sq8_settle_wide(v->cfg, nq, sp, st));
    } else {
        OSK_HIP(launch_sq8_settle(v->cfg, nq, sp, st));
    }
    v->sq8_calls += 1;
    v->sq8w_calls += use_wide ? 1 : 0;
    v->sq6_calls += use6 ? 1 : 0;
    if (probe6) {   // read back asynchronously: a later call folds it (fold_probe), nothing waits here
        OSK_HIP(hipMemcpyAsync(v->h_seg_rebound.p, v->d_seg_rebound.p, sizeof(unsigned long long) * ns,
                               hipMemcpyDeviceToHost, st));
        OSK_HIP(hipEventRecord(v->ev_probe, st));
        v->probe_pending = true;
    }
    return OSK_OK;
}

// The select path (osk_select.hip): exact top-k for any k ≤ OSK_MAX_K, one query at a time.
//   bounds = true: float32 fields through the int8 prefilter copy (bounds → threshold → candidates →
//   exact re-score → top k); bounds = false: exact mode (exact keys → threshold → top k; float32 with the
//   prefilter off, byte vectors).  The candidate buffer holds a whole shard, so nothing overflows and
//   nothing waits on the host.  ws_q / ws_qnorm hold the padded queries (exact mode: the caller's
//   launch_prep_queries; bounds mode: sq8_prep here).
int32_t select_search(osk_view* v, const void* d_queries, int nq, int k, int UP, const uint64_t* const* d_accept,
                      uint64_t* d_shard_keys, int32_t* d_shard_counts, int64_t* d_visited, hipStream_t st,
                      bool bounds) {
    const int S = v->n_shards;
    int64_t total = 0;
    std::vector<int64_t> shard_rows(S, 0);
    for (size_t i = 0; i < v->segs.size(); ++i) {
        total += v->segs[i]->n_rows;
        shard_rows[v->seg_shard[i]] += v->segs[i]->n_rows;
    }
    const int64_t cap = std::max<int64_t>(1, *std::max_element(shard_rows.begin(), shard_rows.end()));
    OSK_REQUIRE(cap < (1ll << 31), "a shard holds < 2^31 rows");
    const int nq_pad = (nq + kMaxNQ - 1) / kMaxNQ * kMaxNQ;
    int u8 = 0;
    if (bounds) {
        int32_t rc = ensure_sq8(v, st);
        if (rc) return rc;
        u8 = v->units8;
        OSK_HIP(v->ws_q8.reserve((size_t)nq_pad * u8 * 16));
        OSK_HIP(v->ws_qc.reserve(sizeof(float4) * nq_pad));
        OSK_HIP(v->ws_flags.reserve(sizeof(int) * nq));
        OSK_HIP(launch_sq8_prep(v->cfg, static_cast<const float*>(d_queries), v->dim, nq, nq_pad, UP, u8,
                                v->ws_q.as<float4>(), v->ws_qnorm.as<float>(), v->ws_q8.p, v->ws_qc.as<float4>(),
                                v->ws_flags.as<int>(), st));
        OSK_HIP(v->ws_sel_lb.reserve(sizeof(uint32_t) * std::max<int64_t>(1, total)));
        OSK_HIP(v->ws_sel_ub.reserve(sizeof(uint32_t) * std::max<int64_t>(1, total)));
    } else {
        if (v->enc == ENC_FLOAT32 && v->sim == SIM_COSINE)
            OSK_HIP(launch_row_norms_f32(v->ws_q.as<float4>(), nq, UP, v->cfg, v->ws_qnorm.as<float>(), st));
        OSK_HIP(v->ws_sel_keys.reserve(sizeof(uint64_t) * std::max<int64_t>(1, total)));
    }
    OSK_HIP(v->ws_sel_state.reserve(sizeof(RadixState) * S));
    OSK_HIP(v->ws_sel_hist.reserve(sizeof(uint32_t) * kSelBins * kSelRep * S));
    OSK_HIP(v->ws_sel_cand.reserve(sizeof(uint64_t) * (size_t)cap * S));
    if (cap > kSelCap) OSK_HIP(v->ws_sel_cand2.reserve(sizeof(uint64_t) * (size_t)cap * S));
    OSK_HIP(v->ws_sel_cnt.reserve(sizeof(int32_t) * std::max(1, v->n_tiles)));
    SelParams p{};
    p.segs = v->d_segs.as<SegDev>();
    p.tiles = v->d_tiles.as<TileDev>();
    p.seg_vrow = v->d_seg_vrow.as<int64_t>();
    p.shard_tile_begin = v->d_shard_tile_begin.as<int32_t>();
    p.tile_coff = v->d_tile_coff.as<int32_t>();
    p.accept = d_accept;
    p.n_tiles = v->n_tiles;
    p.n_shards = S;
    p.n_segs = (int)v->segs.size();
    p.k = k;
    p.sim = v->sim;
    p.dim = v->dim;
    p.units = v->units;
    p.units8 = u8;
    p.enc = v->enc;
    p.exact = bounds ? 0 : 1;
    p.writer = g_tuning.sel_writer.load(std::memory_order_relaxed);
    p.rows8 = v->d_sq8_rows.as<const int4*>();
    p.aux = v->d_sq8_aux.as<const float4*>();
    p.gam = v->sq8_gam;
    p.g2 = v->sq8_g2;
    p.lb = v->ws_sel_lb.as<uint32_t>();
    p.ub = v->ws_sel_ub.as<uint32_t>();
    p.keys = v->ws_sel_keys.as<uint64_t>();
    p.state = v->ws_sel_state.as<RadixState>();
    p.hist = v->ws_sel_hist.as<uint32_t>();
    p.cand = v->ws_sel_cand.as<uint64_t>();
    p.cand2 = v->ws_sel_cand2.as<uint64_t>();
    p.tile_count = v->ws_sel_cnt.as<int32_t>();
    p.cap = (int)cap;
    for (int q = 0; q < nq; ++q) {
        p.q = v->ws_q.as<char>() + (size_t)q * UP * 16;
        p.qnorm = v->ws_qnorm.as<float>() + q;
        p.q8 = v->ws_q8.as<int4>() + (size_t)q * u8;
        p.qc = v->ws_qc.as<float4>() + q;
        p.out_keys = d_shard_keys + (size_t)q * S * k;
        p.out_counts = d_shard_counts + (size_t)q * S;
        p.visited = q == 0 ? reinterpret_cast<unsigned long long*>(d_visited) : nullptr;
        OSK_HIP(launch_select_one(p, v->cfg, st, v->profile && q == 0 ? v->ev0 : nullptr,
                                  v->profile && q == nq - 1 ? v->ev1 : nullptr));
    }
    v->sel_calls += 1;
    return OSK_OK;
}

}  // namespace

namespace osk {

// Lease a workspace slot of `root` for one synchronous host call: a free slot if there is one, else a
// new replica (up to kMaxLeases slots), else wait for a slot to come free.
int32_t lease_view(osk_view* root, ViewLease& out) {
    std::unique_lock<std::mutex> lk(root->lease_mu);
    for (;;) {
        int slot = -1;
        for (size_t i = 0; i < root->lease_busy.size(); ++i)
            if (!root->lease_busy[i]) {
                slot = (int)i;
                break;
            }
        if (slot < 0 && (int)root->lease_busy.size() < osk_view::kMaxLeases) {
            hipStream_t st = nullptr;
            OSK_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
            if (!root->lease_busy.empty()) {   // slots 1..: a replica over the same segments
                std::vector<osk_seg*> segs = root->segs;
                osk_view* v = nullptr;
                int32_t rc = osk_view_create(segs.data(), (int32_t)segs.size(), root->seg_shard.data(),
                                             root->seg_doc_base.data(), root->n_shards, root->shard_index.data(), &v);
                if (rc) {
                    (void)hipStreamDestroy(st);
                    return rc;
                }
                if (!root->holds_refs) {   // a segment's self view: its replicas must not keep it alive
                    v->holds_refs = false;
                    for (osk_seg* sg : segs) sg->refs.fetch_sub(1);
                }
                root->replicas.push_back(v);
            }
            root->lease_streams.push_back(st);
            root->lease_busy.push_back(0);
            slot = (int)root->lease_busy.size() - 1;
        }
        if (slot >= 0) {
            root->lease_busy[slot] = 1;
            out.root = root;
            out.slot = slot;
            out.v = slot == 0 ? root : root->replicas[slot - 1];
            out.st = root->lease_streams[slot];
            return OSK_OK;
        }
        root->lease_cv.wait(lk);
    }
}

ViewLease::~ViewLease() {
    if (!root) return;
    {
        std::lock_guard<std::mutex> lk(root->lease_mu);
        root->lease_busy[slot] = 0;
    }
    root->lease_cv.notify_one();
}

// Every search on a view reuses its workspace.  Calls are serialised by the view mutex on the host,
// but a call on stream B could still overtake a call on stream A on the device, so a search whose
// stream differs from the previous one first waits for everything enqueued on that stream so far
// (an event recorded there now).  Same-stream calls — the common case — pay nothing.  A caller stream
// must therefore stay valid until the next search on the view has been issued (osknn.h).
int32_t order_after_last(osk_view* v, hipStream_t st) {
    if (v->last_stream != nullptr && v->last_stream != st) {
        if (!v->xs_event) OSK_HIP(hipEventCreateWithFlags(&v->xs_event, hipEventDisableTiming));
        OSK_HIP(hipEventRecord(v->xs_event, v->last_stream));
        OSK_HIP(hipStreamWaitEvent(st, v->xs_event, 0));
    }
    v->last_stream = st;
    return OSK_OK;
}

// Core of osk_view_search_device (caller holds the view mutex; device already set).
int32_t view_search_device(osk_view* v, const void* d_queries, int nq, int k,
                           const uint64_t* const* d_accept, uint64_t* d_shard_keys,
                           int32_t* d_shard_counts, int64_t* d_visited, hipStream_t st) {
    OSK_REQUIRE(nq >= 1, "n_queries must be >= 1");
    OSK_REQUIRE(k >= 1 && k <= OSK_MAX_K, "k must be in [1, OSK_MAX_K]");
    OSK_REQUIRE(d_queries && d_shard_keys && d_shard_counts, "null device buffer");
    int32_t rc0 = order_after_last(v, st);
    if (rc0) return rc0;
    static const int kLV[9][2] = {{4, 2}, {8, 2}, {8, 4}, {16, 4}, {16, 8}, {16, 12},
                                  {32, 8}, {64, 8}, {64, 16}};
    const int UP = kLV[v->cfg][0] * kLV[v->cfg][1];
    const int nq_pad = (nq + kMaxNQ - 1) / kMaxNQ * kMaxNQ;
    const int64_t elem = v->enc == ENC_FLOAT32 ? 4 : 1;

    if (v->n_tiles == 0) {   // nothing staged: every shard returns zero hits
        OSK_HIP(hipMemsetAsync(d_shard_keys, 0, sizeof(uint64_t) * nq * v->n_shards * k, st));
        OSK_HIP(hipMemsetAsync(d_shard_counts, 0, sizeof(int32_t) * nq * v->n_shards, st));
        if (d_visited) OSK_HIP(hipMemsetAsync(d_visited, 0, sizeof(int64_t) * v->segs.size(), st));
        return OSK_OK;
    }
    OSK_HIP(v->ws_q.reserve((size_t)nq_pad * UP * 16));
    OSK_HIP(v->ws_qnorm.reserve(sizeof(float) * nq_pad));
    // Path cost model, measured end to end on MI355X, in µs for this view's rows R:
    //   int8 prefilter: the cheaper of its kernels (sq8_narrow_us, sq8_wide_us);
    //   bf16×3, per block of ≤ 256 queries: R·(0.153 + 0.00119·dim) ns + ≈ 325 µs (C3 11.0, C4 27.1, C2 0.63 ms;
    //     fitted to those three, profiles/r02q/c2_batches_*.jsonl, c3_batches_*.jsonl).
    // 96-dim rows stay on the prefilter at any batch, 768-dim rows move to bf16×3 blocks from about 160
    // queries, and small views (C2) from about 128.  sq8_cost_pct scales the prefilter's side (100 = the model).
    const bool sq8_on = v->enc == ENC_FLOAT32 && g_tuning.sq8;
    const bool sq8_ok = sq8_on && k <= kKQ - 4;
    double R = 0.0;
    for (const osk_seg* sg : v->segs) R += (double)sg->n_rows;
    const int u8v = (v->dim + 15) / 16;
    const double sq8_us = sq8_wide_pick(v, nq, d_accept != nullptr) ? sq8_wide_us(R, nq, u8v)
                                                                      : sq8_narrow_us(R, nq, u8v, v->dim);
    const double bf_us = (double)((nq + 255) / 256) * (R * (0.153 + 0.00119 * v->dim) * 1e-3 + 325.0);
    const bool blocks_cheaper = bf_us * 100.0 <= sq8_us * (double)g_tuning.sq8_cost_pct &&
                                !(g_tuning.sq8_wide_force && sq8_wide_pick(v, nq, d_accept != nullptr));
    const bool batched = v->enc == ENC_FLOAT32 && g_tuning.mfma_min_batch > 0 &&
                         nq >= g_tuning.mfma_min_batch && k <= kKC - 4 && (!sq8_ok || blocks_cheaper);
    // k ≤ kKQ − 4: a tile list holds 4 more rows than k, so it rarely overflows past the certificate
    const bool prefilter = !batched && sq8_ok;
    // the select path: k beyond the streaming scans' 64-lane lists, or float32 k beyond the prefilter's
    // lists (its int8 bounds pass reads ¼ of the fp32 scan's bytes)
    const bool select = !batched && !prefilter && (k > kScanMaxK || (sq8_on && k > kKQ - 4 && g_tuning.select_mid_k));
    // queries → padded unit layout (zeros past dim and for the dummy queries of the last launch); the
    // prefilter path does this inside its own fused prep launch (so does the select path's bounds mode)
    if (!prefilter && !(select && sq8_on))
        OSK_HIP(launch_prep_queries(d_queries, (int64_t)v->dim * elem, nq, v->ws_q.p, UP, nq_pad, st));

    if (d_visited) OSK_HIP(hipMemsetAsync(d_visited, 0, sizeof(int64_t) * v->segs.size(), st));

    int32_t rc;
    if ((prefilter || (select && sq8_on)) && (rc = ensure_sq8(v, st)) != OSK_OK) return rc;   // one-time build
    // osk_view_profile(N): every N-th call stamps its scan launches (N = 1: every call); the event stamps cost
    // a few µs of stream time around the stamped launch, so a long timed loop samples instead of stamping all
    v->profile = v->profile_every > 0 && v->profile_tick++ % (uint64_t)v->profile_every == 0;
    if (v->profile && (rc = profile_begin(v, st, batched)) != OSK_OK) return rc;
    if (select) {
        rc = select_search(v, d_queries, nq, k, UP, d_accept, d_shard_keys, d_shard_counts, d_visited, st, sq8_on);
        if (rc == OSK_OK) rc = profile_end(v, st, false);
    } else if (prefilter) {
        rc = sq8_search(v, d_queries, nq, k, UP, d_accept, d_shard_keys, d_shard_counts, d_visited, st);
    } else if (batched) {
        // |q|² in the device lane layout: approx transforms, the re-score (COSINE) and the bound
        OSK_HIP(launch_row_norms_f32(v->ws_q.as<float4>(), nq, UP, v->cfg, v->ws_qnorm.as<float>(), st));
        rc = batched_search(v, nq, k, UP, d_accept, d_shard_keys, d_shard_counts, d_visited, st);
    } else {
        rc = stream_search(v, v->ws_q.p, v->ws_qnorm.p, nq, k, UP, d_accept, d_shard_keys, d_shard_counts,
                           d_visited, st);
    }
    if (rc) return rc;
    return OSK_OK;
}

}  // namespace osk

extern "C" {

int32_t osk_view_search_device(osk_view* view, const void* d_queries, int32_t n_queries, int32_t k,
                               const uint64_t* const* d_accept, uint64_t* d_shard_keys,
                               int32_t* d_shard_counts, int64_t* d_visited, void* stream) {
    OSK_GUARD_BEGIN
    clear_error();
    OSK_REQUIRE(view != nullptr, "view is null");
    int32_t rc = check_device(view->device);
    if (rc) return rc;
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : device_stream(view->device);
    std::lock_guard<std::mutex> lk(view->mu);
    return view_search_device(view, d_queries, n_queries, k, d_accept, d_shard_keys, d_shard_counts,
                              d_visited, st);
    OSK_GUARD_END
}

int32_t osk_merge_device(int32_t device, const uint64_t* d_shard_keys, const int32_t* d_shard_counts,
                         const int32_t* d_shard_index, int32_t n_queries, int32_t n_shards, int32_t k,
                         int32_t from, int32_t size, float* d_scores, int32_t* d_docs,
                         int32_t* d_shard_out, int32_t* d_count, int64_t* d_total_hits,
                         float* d_max_score, void* stream) {
    OSK_GUARD_BEGIN
    clear_error();
    OSK_REQUIRE(n_queries >= 1 && n_shards >= 1, "n_queries and n_shards must be >= 1");
    OSK_REQUIRE(k >= 1 && k <= OSK_MAX_K, "k must be in [1, OSK_MAX_K]");
    OSK_REQUIRE(from >= 0 && size >= 1 && (int64_t)from + size <= 100000, "bad from/size");
    OSK_REQUIRE(d_shard_keys && d_shard_counts && d_shard_index && d_scores && d_docs && d_shard_out &&
                    d_count && d_total_hits && d_max_score,
                "null device buffer");
    int32_t rc = check_device(device);
    if (rc) return rc;
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : device_stream(device);
    OSK_HIP(launch_coord_reduce(d_shard_keys, d_shard_counts, d_shard_index, n_queries, 1, n_shards, k,
                               from, size, d_scores, d_docs, d_shard_out, d_count, d_total_hits,
                               d_max_score, st));
    return OSK_OK;
    OSK_GUARD_END
}

int32_t osk_merge_device_ranked(int32_t device, const uint64_t* d_keys, int32_t n_ranks,
                                int32_t shards_per_rank, const int32_t* d_shard_index, int32_t n_queries,
                                int32_t k, int32_t from, int32_t size, float* d_scores, int32_t* d_docs,
                                int32_t* d_shard_out, int32_t* d_count, int64_t* d_total_hits,
                                float* d_max_score, void* stream) {
    OSK_GUARD_BEGIN
    clear_error();
    OSK_REQUIRE(n_queries >= 1 && n_ranks >= 1 && shards_per_rank >= 1,
                "n_queries, n_ranks and shards_per_rank must be >= 1");
    OSK_REQUIRE(k >= 1 && k <= OSK_MAX_K, "k must be in [1, OSK_MAX_K]");
    OSK_REQUIRE(from >= 0 && size >= 1 && (int64_t)from + size <= 100000, "bad from/size");
    OSK_REQUIRE(d_keys && d_shard_index && d_scores && d_docs && d_shard_out && d_count && d_total_hits &&
                    d_max_score,
                "null device buffer");
    int32_t rc = check_device(device);
    if (rc) return rc;
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : device_stream(device);
    OSK_HIP(launch_coord_reduce(d_keys, nullptr, d_shard_index, n_queries, n_ranks, shards_per_rank, k, from,
                               size, d_scores, d_docs, d_shard_out, d_count, d_total_hits, d_max_score, st));
    return OSK_OK;
    OSK_GUARD_END
}

// Scan-kernel timing for bench.py: enable, then read the mean duration of the scan launches of
// each search call (all query chunks of one call together) since enabling.
int32_t osk_view_profile(osk_view* v, int32_t enable) {
    OSK_GUARD_BEGIN
    OSK_REQUIRE(v != nullptr, "view is null");
    int32_t rc = check_device(v->device);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(v->mu);
    if (enable && !v->ev_start[0]) {
        for (int i = 0; i < osk_view::kEvRing; ++i) {
            OSK_HIP(hipEventCreate(&v->ev_start[i]));
            OSK_HIP(hipEventCreate(&v->ev_stop[i]));
        }
    }
    OSK_REQUIRE(enable >= 0, "enable must be >= 0");
    for (int i = 0; i < osk_view::kEvRing; ++i) v->ev_pending[i] = false;
    v->profile = false;
    v->profile_every = enable;
    v->profile_tick = 0;
    v->scan_ms = 0.0;
    v->scan_calls = 0;
    v->ev_next = 0;
    return OSK_OK;
    OSK_GUARD_END
}

// Test/debug only: copy an internal workspace buffer of the last search to host memory.
int32_t osk_view_debug_copy(osk_view* v, const char* name, void* host, int64_t bytes) {
    OSK_GUARD_BEGIN
#ifndef OSK_TESTING
    (void)v; (void)name; (void)host; (void)bytes;
    set_error("osk_view_debug_copy exists only in the testing build (libosknn_testing.so)");
    return OSK_ERR_UNSUPPORTED;
#else
    OSK_REQUIRE(v && name && host && bytes >= 0, "null argument");
    int32_t rc = check_device(v->device);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(v->mu);
    const std::string n(name);
    const DevBuf* b = n == "akeys" ? &v->ws_akeys : n == "cand_a" ? &v->ws_cand_a : n == "flags" ? &v->ws_flags
                    : n == "qsplit" ? &v->ws_qsplit : n == "qnorm" ? &v->ws_qnorm
                    : n == "sq8cand" ? &v->ws_sq8cand : n == "sq8lb" ? &v->ws_sq8lb : n == "qc" ? &v->ws_qc
                    : n == "settle_trace" ? &v->ws_trace
                    : nullptr;
    OSK_REQUIRE(b != nullptr, "unknown buffer");
    OSK_REQUIRE((size_t)bytes <= b->cap, "bytes exceed the buffer");
    OSK_HIP(hipDeviceSynchronize());   // the last search may be on any stream
    OSK_HIP(hipMemcpy(host, b->p, bytes, hipMemcpyDeviceToHost));
    return OSK_OK;
#endif
    OSK_GUARD_END
}

// The view and every replica its host entries leased (slots): counters are summed over them.
static std::vector<osk_view*> slot_views(osk_view* v) {
    std::lock_guard<std::mutex> lk(v->lease_mu);
    std::vector<osk_view*> out{v};
    out.insert(out.end(), v->replicas.begin(), v->replicas.end());
    return out;
}

int32_t osk_view_stats(osk_view* v, int64_t* batched_calls, int64_t* fallback_queries) {
    OSK_GUARD_BEGIN
    OSK_REQUIRE(v != nullptr && batched_calls && fallback_queries, "null argument");
    *batched_calls = *fallback_queries = 0;
    for (osk_view* s : slot_views(v)) {
        std::lock_guard<std::mutex> lk(s->mu);
        *batched_calls += s->mfma_calls;
        *fallback_queries += s->mfma_fallback_queries;
    }
    return OSK_OK;
    OSK_GUARD_END
}

int32_t osk_view_counter(osk_view* v, const char* name, int64_t* value) {
    OSK_GUARD_BEGIN
    OSK_REQUIRE(v != nullptr && name != nullptr && value != nullptr, "null argument");
    int32_t rc = check_device(v->device);
    if (rc) return rc;
    const std::string n(name);
    if (n == "host_slots") {   // workspace slots the host entries have leased so far (1 + replicas)
        std::lock_guard<std::mutex> lk(v->lease_mu);
        *value = (int64_t)v->lease_busy.size();
        return OSK_OK;
    }
    if (n == "host_batches" || n == "host_batched_requests") {   // opportunistic batching of host calls
        std::lock_guard<std::mutex> lk(v->batcher.mu);
        *value = n == "host_batches" ? v->batcher.batches : v->batcher.requests;
        return OSK_OK;
    }
    if (n == "sq8_slices") {
        std::lock_guard<std::mutex> lk(v->mu);
        *value = v->n_slices;
        return OSK_OK;
    }
    if (n == "mfma_full_tiles") {   // (root view only)
        std::lock_guard<std::mutex> lk(v->mu);
        unsigned long long c = 0;
        if (v->d_mfma_full.p) {
            OSK_HIP(hipDeviceSynchronize());
            OSK_HIP(hipMemcpy(&c, v->d_mfma_full.p, sizeof(c), hipMemcpyDeviceToHost));
        }
        *value = (int64_t)c;
        return OSK_OK;
    }
    const bool dev = n == "sq8_fallback_queries" || n == "sq8_rescored_rows" || n == "sq8_exact_tiles" ||
                     n == "sq6_rebound_rows" || n == "sq8_wide_events" || n == "sq8_wide_pairs" ||
                     n == "sq8_wide_wait_cycles" || n == "sq8_wide_slow_steps" || n == "sq8_wide_loop_cycles" ||
                     n == "sq8_wide_slow_cycles" || n == "sq8_wide_drain_cycles" ||
                     n == "sq6_rebound_gathered_rows" || n == "sq6_rebound_passes" ||
                     n == "sq6_rebound_max_wg_cycles" || n == "sq8_rows_total_cycles" || n == "sq8_rows_setup_cycles" ||
                     n == "sq8_rows_quarter_end_cycles" || n == "sq8_rows_first_wait_cycles" ||
                     n == "sq8_rows_setup_barrier_cycles" || n == "sq8_rows_setup_fragment_cycles";
    OSK_REQUIRE(dev || n == "mfma_calls" || n == "mfma_fallback_queries" || n == "sq8_calls" || n == "sq6_calls" ||
                    n == "select_calls" || n == "sq8_wide_calls",
                "unknown counter: " + n);
    // summed over the view and the replicas its host entries leased
    int64_t sum = 0;
    for (osk_view* s : slot_views(v)) {
        std::lock_guard<std::mutex> lk(s->mu);
        if (dev) {
            if (!s->d_counters.p) continue;
            unsigned long long c[24];
            OSK_HIP(hipDeviceSynchronize());   // the last search may be on any stream
            OSK_HIP(hipMemcpy(c, s->d_counters.p, sizeof(c), hipMemcpyDeviceToHost));
            // [4] … [8]: the wide kernel's insertion events, quick-test passes, wave 0's shader clocks in the
            // step loop's waits [6] and whole loop [8], and the wave-steps that took the slow path [7] (testing build)
            sum += (int64_t)(n == "sq8_fallback_queries" ? c[0] : n == "sq8_rescored_rows" ? c[1]
                             : n == "sq8_exact_tiles" ? c[2] : n == "sq6_rebound_rows" ? c[3]
                             : n == "sq8_wide_events" ? c[4] : n == "sq8_wide_pairs" ? c[5]
                             : n == "sq8_wide_wait_cycles" ? c[6] : n == "sq8_wide_slow_steps" ? c[7]
                             : n == "sq8_wide_loop_cycles" ? c[8] : n == "sq8_wide_slow_cycles" ? c[9]
                             : n == "sq8_wide_drain_cycles" ? c[10] : n == "sq6_rebound_gathered_rows" ? c[11]
                             : n == "sq6_rebound_passes" ? c[12] : n == "sq6_rebound_max_wg_cycles" ? c[13]
                             // [16] … [19]: sq8_wide_rows, wave 0's shader clocks per workgroup summed: the whole
                             // kernel, its setup (to the first quarter), the quarter ends (publish, barriers, drain,
                             // flush, next constants), the waits for each quarter's first group (testing build)
                             : n == "sq8_rows_total_cycles" ? c[16] : n == "sq8_rows_setup_cycles" ? c[17]
                             : n == "sq8_rows_quarter_end_cycles" ? c[18] : n == "sq8_rows_first_wait_cycles" ? c[19]
                             : n == "sq8_rows_setup_barrier_cycles" ? c[20] : c[21]);
        } else {
            sum += n == "mfma_calls" ? s->mfma_calls : n == "mfma_fallback_queries" ? s->mfma_fallback_queries
                 : n == "sq8_calls" ? s->sq8_calls : n == "sq6_calls" ? s->sq6_calls
                 : n == "sq8_wide_calls" ? s->sq8w_calls : s->sel_calls;
        }
    }
    *value = sum;
    return OSK_OK;
    OSK_GUARD_END
}

int32_t osk_view_scan_time(osk_view* v, double* total_ms, int64_t* calls) {
    OSK_GUARD_BEGIN
    OSK_REQUIRE(v != nullptr && total_ms && calls, "null argument");
    int32_t rc = check_device(v->device);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(v->mu);
    for (int i = 0; i < osk_view::kEvRing; ++i) {
        rc = profile_fold(v, i);
        if (rc) return rc;
    }
    *total_ms = v->scan_ms;
    *calls = v->scan_calls;
    return OSK_OK;
    OSK_GUARD_END
}

// Host-buffer search + coordinator merge on one device (synchronous).
static int32_t view_search_host(osk_view* v, const void* queries, int32_t n_queries, int32_t k, int32_t from,
                                int32_t size, const uint64_t* const* accept, float* out_scores,
                                int32_t* out_docs, int32_t* out_shard_index, int32_t* out_count,
                                int64_t* out_total_hits, float* out_max_score) {
    OSK_GUARD_BEGIN
    clear_error();
    OSK_REQUIRE(v != nullptr && queries != nullptr, "null argument");
    OSK_REQUIRE(out_scores && out_docs && out_shard_index && out_count && out_total_hits && out_max_score,
                "null output");
    OSK_REQUIRE(n_queries >= 1, "n_queries must be >= 1");
    OSK_REQUIRE(from >= 0 && size >= 1, "bad from/size");
    int32_t rc = check_device(v->device);
    if (rc) return rc;
    ViewLease lease;   // a workspace slot (this view or a replica) and its stream, for this call
    rc = lease_view(v, lease);
    if (rc) return rc;
    v = lease.v;
    hipStream_t st = lease.st;
    std::lock_guard<std::mutex> lk(v->mu);
    rc = order_after_last(v, st);
    if (rc) return rc;
    const int nq = n_queries, S = v->n_shards, ns = (int)v->segs.size();
    const int64_t elem = v->enc == ENC_FLOAT32 ? 4 : 1;
    const size_t qbytes = (size_t)nq * v->dim * elem;
    CallTimer timer;
    if ((rc = timer.begin(v, st)) != OSK_OK) return rc;

    // accept bitsets → device
    const uint64_t* const* d_acc = nullptr;
    bool any_bits = false;   // no leaf with a bitset = no filter (the unfiltered scan instances)
    for (int i = 0; accept && i < ns; ++i) any_bits |= accept[i] != nullptr;
    if (any_bits) {
        size_t words = 0;
        for (int i = 0; i < ns; ++i)
            if (accept[i]) words += (size_t)(v->segs[i]->max_doc + 63) / 64;
        OSK_HIP(v->ws_accept.reserve(std::max<size_t>(8, words * 8)));
        OSK_HIP(v->ws_accept_ptrs.reserve(sizeof(void*) * ns));
        // the pointer table is staged in the view's pinned buffer: it is the source of an async copy and
        // must outlive it (the stream is synchronised only at the end of the call)
        OSK_HIP(v->h_accept_tab.reserve(sizeof(void*) * ns));
        const uint64_t** ptrs = static_cast<const uint64_t**>(v->h_accept_tab.p);
        size_t off = 0;
        for (int i = 0; i < ns; ++i) {
            ptrs[i] = nullptr;
            if (!accept[i]) continue;
            const size_t w = (size_t)(v->segs[i]->max_doc + 63) / 64;
            ptrs[i] = v->ws_accept.as<uint64_t>() + off;
            OSK_HIP(hipMemcpyAsync(const_cast<uint64_t*>(ptrs[i]), accept[i], w * 8,
                                   hipMemcpyHostToDevice, st));
            off += w;
        }
        OSK_HIP(hipMemcpyAsync(v->ws_accept_ptrs.p, ptrs, sizeof(void*) * ns, hipMemcpyHostToDevice, st));
        d_acc = v->ws_accept_ptrs.as<const uint64_t*>();
    }
    OSK_HIP(v->ws_qin.reserve(std::max<size_t>(16, qbytes)));
    OSK_HIP(hipMemcpyAsync(v->ws_qin.p, queries, qbytes, hipMemcpyHostToDevice, st));
    OSK_HIP(v->ws_keys.reserve(sizeof(uint64_t) * (size_t)nq * S * k));
    OSK_HIP(v->ws_counts.reserve(sizeof(int32_t) * (size_t)nq * S));
    rc = view_search_device(v, v->ws_qin.p, nq, k, d_acc, v->ws_keys.as<uint64_t>(),
                            v->ws_counts.as<int32_t>(), nullptr, st);
    if (rc) return rc;
    // outputs: scores f32 | docs i32 | shard i32 | count i32 | total i64 | max f32
    const size_t n_out = (size_t)nq * size;
    const size_t b_sc = n_out * 4, b_doc = n_out * 4, b_sh = n_out * 4, b_cnt = nq * 4,
                 b_tot = nq * 8, b_max = nq * 4;
    const size_t o_sc = 0, o_doc = o_sc + b_sc, o_sh = o_doc + b_doc, o_cnt = o_sh + b_sh,
                 o_tot = (o_cnt + b_cnt + 7) / 8 * 8, o_max = o_tot + b_tot,
                 total_b = o_max + b_max;
    OSK_HIP(v->ws_out.reserve(total_b));
    char* ob = v->ws_out.as<char>();
    OSK_HIP(launch_coord_reduce(v->ws_keys.as<uint64_t>(), v->ws_counts.as<int32_t>(),
                               v->d_shard_index.as<int32_t>(), nq, 1, S, k, from, size,
                               reinterpret_cast<float*>(ob + o_sc), reinterpret_cast<int32_t*>(ob + o_doc),
                               reinterpret_cast<int32_t*>(ob + o_sh), reinterpret_cast<int32_t*>(ob + o_cnt),
                               reinterpret_cast<int64_t*>(ob + o_tot), reinterpret_cast<float*>(ob + o_max),
                               st));
    OSK_HIP(v->h_stage.reserve(total_b));
    OSK_HIP(hipMemcpyAsync(v->h_stage.p, ob, total_b, hipMemcpyDeviceToHost, st));
    if ((rc = timer.end()) != OSK_OK) return rc;
    OSK_HIP(hipStreamSynchronize(st));
    if ((rc = timer.publish()) != OSK_OK) return rc;
    const char* hb = static_cast<const char*>(v->h_stage.p);
    std::memcpy(out_scores, hb + o_sc, b_sc);
    std::memcpy(out_docs, hb + o_doc, b_doc);
    std::memcpy(out_shard_index, hb + o_sh, b_sh);
    std::memcpy(out_count, hb + o_cnt, b_cnt);
    std::memcpy(out_total_hits, hb + o_tot, b_tot);
    std::memcpy(out_max_score, hb + o_max, b_max);
    return OSK_OK;
    OSK_GUARD_END
}

static int32_t seg_search_host(osk_seg* seg, const void* queries, int32_t n_queries, int32_t k,
                               const uint64_t* accept_bits, float* out_scores, int32_t* out_docs,
                               int32_t* out_count, int64_t* out_visited) {
    OSK_GUARD_BEGIN
    clear_error();
    OSK_REQUIRE(seg != nullptr && queries != nullptr, "null argument");
    OSK_REQUIRE(out_scores && out_docs && out_count, "null output");
    OSK_REQUIRE(n_queries >= 1, "n_queries must be >= 1");
    OSK_REQUIRE(k >= 1 && k <= OSK_MAX_K, "k must be in [1, OSK_MAX_K]");
    int32_t rc = check_device(seg->device);
    if (rc) return rc;
    osk_view* v;
    {
        std::lock_guard<std::mutex> lk(seg->mu);
        if (!seg->self_view) {
            osk_seg* one[1] = {seg};
            rc = osk_view_create(one, 1, nullptr, nullptr, 1, nullptr, &seg->self_view);
            if (rc) return rc;
            // owned by the segment: it must not keep the segment alive
            seg->self_view->holds_refs = false;
            seg->refs.fetch_sub(1);
        }
        v = seg->self_view;
    }
    (void)hipSetDevice(seg->device);
    ViewLease lease;   // a workspace slot (the self view or a replica) and its stream, for this call
    rc = lease_view(v, lease);
    if (rc) return rc;
    v = lease.v;
    hipStream_t st = lease.st;
    std::lock_guard<std::mutex> lk(v->mu);
    rc = order_after_last(v, st);
    if (rc) return rc;
    const int nq = n_queries;
    const int64_t elem = seg->enc == ENC_FLOAT32 ? 4 : 1;
    const size_t qbytes = (size_t)nq * seg->dim * elem;
    CallTimer timer;
    if ((rc = timer.begin(v, st)) != OSK_OK) return rc;
    const uint64_t* const* d_acc = nullptr;
    if (accept_bits) {
        const size_t w = (size_t)(seg->max_doc + 63) / 64;
        OSK_HIP(v->ws_accept.reserve(std::max<size_t>(8, w * 8)));
        OSK_HIP(v->ws_accept_ptrs.reserve(sizeof(void*)));
        if (w) OSK_HIP(hipMemcpyAsync(v->ws_accept.p, accept_bits, w * 8, hipMemcpyHostToDevice, st));
        // the source of the async copy must outlive it: a view member (the call synchronises below)
        v->h_accept_ptr = v->ws_accept.as<uint64_t>();
        OSK_HIP(hipMemcpyAsync(v->ws_accept_ptrs.p, &v->h_accept_ptr, sizeof(void*), hipMemcpyHostToDevice, st));
        d_acc = v->ws_accept_ptrs.as<const uint64_t*>();
    }
    OSK_HIP(v->ws_qin.reserve(std::max<size_t>(16, qbytes)));
    OSK_HIP(hipMemcpyAsync(v->ws_qin.p, queries, qbytes, hipMemcpyHostToDevice, st));
    OSK_HIP(v->ws_keys.reserve(sizeof(uint64_t) * (size_t)nq * k));
    OSK_HIP(v->ws_counts.reserve(sizeof(int32_t) * (size_t)nq));
    OSK_HIP(v->ws_visited.reserve(sizeof(int64_t)));
    rc = view_search_device(v, v->ws_qin.p, nq, k, d_acc, v->ws_keys.as<uint64_t>(),
                            v->ws_counts.as<int32_t>(), v->ws_visited.as<int64_t>(), st);
    if (rc) return rc;
    const size_t kb = sizeof(uint64_t) * (size_t)nq * k, cb = sizeof(int32_t) * nq;
    OSK_HIP(v->h_stage.reserve(kb + cb + 8));
    char* hb = static_cast<char*>(v->h_stage.p);
    OSK_HIP(hipMemcpyAsync(hb, v->ws_keys.p, kb, hipMemcpyDeviceToHost, st));
    OSK_HIP(hipMemcpyAsync(hb + kb, v->ws_counts.p, cb, hipMemcpyDeviceToHost, st));
    OSK_HIP(hipMemcpyAsync(hb + kb + cb, v->ws_visited.p, 8, hipMemcpyDeviceToHost, st));
    if ((rc = timer.end()) != OSK_OK) return rc;
    OSK_HIP(hipStreamSynchronize(st));
    if ((rc = timer.publish()) != OSK_OK) return rc;
    const uint64_t* keys = reinterpret_cast<const uint64_t*>(hb);
    const int32_t* cnt = reinterpret_cast<const int32_t*>(hb + kb);
    int64_t visited;
    std::memcpy(&visited, hb + kb + cb, 8);
    for (int q = 0; q < nq; ++q) {
        out_count[q] = cnt[q];
        for (int i = 0; i < k; ++i) {
            const uint64_t key = keys[(size_t)q * k + i];
            const size_t o = (size_t)q * k + i;
            if (i < cnt[q]) {
                out_scores[o] = key_score(key);
                out_docs[o] = key_doc(key);
            } else {
                out_scores[o] = -__builtin_inff();
                out_docs[o] = 0x7FFFFFFF;
            }
        }
        if (out_visited) out_visited[q] = visited;
    }
    return OSK_OK;
    OSK_GUARD_END
}

// Opportunistic batching of concurrent host calls ("batches concurrent single-query
// calls opportunistically").  A call queues its request on the view; while fewer than host_batch_leaders
// batches are in flight, a waiting caller becomes a leader, takes the compatible requests queued so far
// (FIFO, same k / from / size, no filter, ≤ 32 queries) and runs them as ONE batched search (the int8
// MFMA prefilter reads the corpus once for all of them), then hands every request its rows (at most
// host_batch_leaders batches in flight per view).  No
// artificial delay: requests batch up only while the device is busy with earlier ones.  Results are
// identical to unbatched calls (every path is exact).
}  // extern "C"

namespace {

constexpr int kBatchMaxQueries = 32;

struct BatchReq {
    const void* queries;
    int nq, k, from, size;
    float* sc;
    int32_t* docs;
    int32_t* shard;
    int32_t* cnt;
    int64_t* tot;
    float* mx;
    int64_t* visited;
    int32_t rc = OSK_OK;
    std::string err;
    bool done = false;
    int64_t device_ns = -1;   // the serving launch chain's device time (call_timing) ...
    int32_t shared = 0;       // ... and how many requests it served
};

// run `fn(batch, total_queries)` as a leader whenever possible until `me` is done
template <class Fn>
int32_t batched_call(osk_view* root, BatchReq& me, Fn&& fn) {
    auto& B = root->batcher;
    std::unique_lock<std::mutex> lk(B.mu);
    B.queue.push_back(&me);
    while (!me.done) {
        if (!B.queue.empty() && B.leaders < (int)g_tuning.host_batch_leaders) {
            std::vector<BatchReq*> batch;
            int total = 0;
            const BatchReq* f = static_cast<const BatchReq*>(B.queue.front());
            for (auto it = B.queue.begin(); it != B.queue.end();) {
                BatchReq* r = static_cast<BatchReq*>(*it);
                if (r->k == f->k && r->from == f->from && r->size == f->size && total + r->nq <= kBatchMaxQueries) {
                    batch.push_back(r);
                    total += r->nq;
                    it = B.queue.erase(it);
                } else {
                    ++it;
                }
            }
            ++B.leaders;
            lk.unlock();
            int32_t rc;
            t_call_ns = -1;
            try {   // the batch's requests must always be completed, whatever happens
                rc = fn(batch, total);
            } catch (const std::bad_alloc&) {
                set_error("host allocation failed");
                rc = OSK_ERR_OOM;
            } catch (...) {
                set_error("batched search failed");
                rc = OSK_ERR_INVALID;
            }
            const std::string err = rc ? std::string(osk_last_error()) : std::string();
            lk.lock();
            for (BatchReq* r : batch) {
                r->rc = rc;
                r->err = err;
                r->device_ns = t_call_ns;
                r->shared = t_call_ns >= 0 ? (int32_t)batch.size() : 0;
                r->done = true;
            }
            --B.leaders;
            B.batches += 1;
            B.requests += (int64_t)batch.size();
            B.cv.notify_all();
        } else {
            B.cv.wait(lk);
        }
    }
    t_call_ns = me.device_ns;
    t_call_shared = me.shared;
    if (me.rc) set_error("batched search: " + me.err);
    return me.rc;
}

}  // namespace

extern "C" {

int32_t osk_view_search(osk_view* v, const void* queries, int32_t n_queries, int32_t k, int32_t from,
                        int32_t size, const uint64_t* const* accept, float* out_scores,
                        int32_t* out_docs, int32_t* out_shard_index, int32_t* out_count,
                        int64_t* out_total_hits, float* out_max_score) {
    OSK_GUARD_BEGIN
    clear_error();
    OSK_REQUIRE(v != nullptr && queries != nullptr, "null argument");
    bool any_bits = false;
    for (int i = 0; accept && i < (int)v->segs.size(); ++i) any_bits |= accept[i] != nullptr;
    if (any_bits || !g_tuning.host_batching || n_queries < 1 || n_queries > kBatchMaxQueries)
        return view_search_host(v, queries, n_queries, k, from, size, accept, out_scores, out_docs, out_shard_index,
                                out_count, out_total_hits, out_max_score);
    BatchReq me{queries, n_queries, k, from, size, out_scores, out_docs, out_shard_index, out_count,
                out_total_hits, out_max_score, nullptr};
    const size_t qrow = (size_t)v->dim * (v->enc == ENC_FLOAT32 ? 4 : 1);
    return batched_call(v, me, [&](const std::vector<BatchReq*>& batch, int total) -> int32_t {
        if (batch.size() == 1) {
            BatchReq* r = batch[0];
            return view_search_host(v, r->queries, r->nq, r->k, r->from, r->size, nullptr, r->sc, r->docs, r->shard,
                                    r->cnt, r->tot, r->mx);
        }
        const int sz = batch[0]->size;
        std::vector<char> q((size_t)total * qrow);
        std::vector<float> sc((size_t)total * sz), mx(total);
        std::vector<int32_t> dc((size_t)total * sz), sh((size_t)total * sz), cnt(total);
        std::vector<int64_t> tot(total);
        int off = 0;
        for (BatchReq* r : batch) {
            std::memcpy(q.data() + (size_t)off * qrow, r->queries, (size_t)r->nq * qrow);
            off += r->nq;
        }
        const int32_t rc = view_search_host(v, q.data(), total, batch[0]->k, batch[0]->from, sz, nullptr, sc.data(),
                                            dc.data(), sh.data(), cnt.data(), tot.data(), mx.data());
        if (rc) return rc;
        off = 0;
        for (BatchReq* r : batch) {
            const size_t o = (size_t)off * sz, n = (size_t)r->nq * sz;
            std::memcpy(r->sc, sc.data() + o, n * 4);
            std::memcpy(r->docs, dc.data() + o, n * 4);
            std::memcpy(r->shard, sh.data() + o, n * 4);
            std::memcpy(r->cnt, cnt.data() + off, (size_t)r->nq * 4);
            std::memcpy(r->tot, tot.data() + off, (size_t)r->nq * 8);
            std::memcpy(r->mx, mx.data() + off, (size_t)r->nq * 4);
            off += r->nq;
        }
        return OSK_OK;
    });
    OSK_GUARD_END
}

// [L] KnnVectorsReader.search on one segment (host buffers, synchronous).
int32_t osk_seg_search(osk_seg* seg, const void* queries, int32_t n_queries, int32_t k,
                       const uint64_t* accept_bits, float* out_scores, int32_t* out_docs,
                       int32_t* out_count, int64_t* out_visited) {
    OSK_GUARD_BEGIN
    clear_error();
    OSK_REQUIRE(seg != nullptr && queries != nullptr, "null argument");
    if (accept_bits || !g_tuning.host_batching || n_queries < 1 || n_queries > kBatchMaxQueries)
        return seg_search_host(seg, queries, n_queries, k, accept_bits, out_scores, out_docs, out_count, out_visited);
    osk_view* root;
    {
        std::lock_guard<std::mutex> lk(seg->mu);
        if (!seg->self_view) {
            osk_seg* one[1] = {seg};
            int32_t rc = osk_view_create(one, 1, nullptr, nullptr, 1, nullptr, &seg->self_view);
            if (rc) return rc;
            seg->self_view->holds_refs = false;   // owned by the segment: must not keep it alive
            seg->refs.fetch_sub(1);
        }
        root = seg->self_view;
    }
    BatchReq me{queries, n_queries, k, 0, k, out_scores, out_docs, nullptr, out_count, nullptr, nullptr, out_visited};
    const size_t qrow = (size_t)seg->dim * (seg->enc == ENC_FLOAT32 ? 4 : 1);
    return batched_call(root, me, [&](const std::vector<BatchReq*>& batch, int total) -> int32_t {
        if (batch.size() == 1) {
            BatchReq* r = batch[0];
            return seg_search_host(seg, r->queries, r->nq, r->k, nullptr, r->sc, r->docs, r->cnt, r->visited);
        }
        const int kk = batch[0]->k;
        std::vector<char> q((size_t)total * qrow);
        std::vector<float> sc((size_t)total * kk);
        std::vector<int32_t> dc((size_t)total * kk), cnt(total);
        std::vector<int64_t> vis(total);
        int off = 0;
        for (BatchReq* r : batch) {
            std::memcpy(q.data() + (size_t)off * qrow, r->queries, (size_t)r->nq * qrow);
            off += r->nq;
        }
        const int32_t rc = seg_search_host(seg, q.data(), total, kk, nullptr, sc.data(), dc.data(), cnt.data(), vis.data());
        if (rc) return rc;
        off = 0;
        for (BatchReq* r : batch) {
            const size_t o = (size_t)off * kk, n = (size_t)r->nq * kk;
            std::memcpy(r->sc, sc.data() + o, n * 4);
            std::memcpy(r->docs, dc.data() + o, n * 4);
            std::memcpy(r->cnt, cnt.data() + off, (size_t)r->nq * 4);
            if (r->visited) std::memcpy(r->visited, vis.data() + off, (size_t)r->nq * 8);
            off += r->nq;
        }
        return OSK_OK;
    });
    OSK_GUARD_END
}

int32_t osk_last_call_device_ns(int64_t* device_ns, int32_t* shared_by) {
    OSK_GUARD_BEGIN
    OSK_REQUIRE(device_ns != nullptr, "null argument");
    *device_ns = t_call_ns;
    if (shared_by) *shared_by = t_call_shared;
    return OSK_OK;
    OSK_GUARD_END
}

}  // extern "C"
