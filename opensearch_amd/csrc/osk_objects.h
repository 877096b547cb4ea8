// osk_objects.h — the host-side object model of libosknn (osk_seg, osk_view, osk_comm helpers) shared
// by the C-ABI translation units (osk_api.hip, osk_comm.hip).  Not part of the public ABI.
//
//   osk_seg   one segment's vector field in HBM (rows padded to 16-byte units, optional row norms,
//             optional ord→doc map, and the derived copies the fast paths read: the int8 prefilter
//             copy + bound terms, its MFMA-tiled twin, the bf16 hi/lo split).  Reference counted:
//             the reader holds one reference ([L] KnnVectorsFormat.fieldsReader … close()), every view
//             that groups it holds another, so a segment merged away under a live view stays valid
//             until the view is released (NRT refresh churn, S/index/engine/InternalEngine.java:584-589).
//   osk_view  the segments of one or more shards on one device plus the scan's tile table and a
//             workspace.  A shard's exact top-k = per-leaf exact top-k merged by (score, doc)
//             ([L] AbstractKnnVectorQuery.rewrite, driven from
//             S/search/internal/ContextIndexSearcher.java:203-218).
#pragma once
#include <hip/hip_runtime.h>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/osknn.h"
#include "osk_internal.h"

namespace osk {

void set_error(const std::string& msg);
void clear_error();

#define OSK_HIP(call)                                                                          \
    do {                                                                                       \
        hipError_t e_ = (call);                                                                \
        if (e_ != hipSuccess) {                                                                \
            ::osk::set_error(std::string(#call) + ": " + hipGetErrorString(e_));               \
            return OSK_ERR_DEVICE;                                                             \
        }                                                                                      \
    } while (0)

#define OSK_REQUIRE(cond, msg)                                                                 \
    do {                                                                                       \
        if (!(cond)) {                                                                         \
            ::osk::set_error(msg);                                                             \
            return OSK_ERR_INVALID;                                                            \
        }                                                                                      \
    } while (0)

#define OSK_GUARD_BEGIN try {
#define OSK_GUARD_END                                                                          \
    }                                                                                          \
    catch (const std::bad_alloc&) {                                                            \
        ::osk::set_error("host allocation failed");                                            \
        return OSK_ERR_OOM;                                                                    \
    }                                                                                          \
    catch (const std::exception& ex) {                                                         \
        ::osk::set_error(ex.what());                                                           \
        return OSK_ERR_INVALID;                                                                \
    }                                                                                          \
    catch (...) {                                                                              \
        ::osk::set_error("unknown exception");                                                 \
        return OSK_ERR_INVALID;                                                                \
    }

// devices and streams
int device_count_cached();
int32_t check_device(int device);      // also makes `device` current on this thread
hipStream_t device_stream(int device);  // the library's own non-blocking stream of a device

// device buffer that grows on demand (never inside a timed/captured call once warmed)
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
    hipError_t reserve(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) {
            (void)hipFree(p);
            p = nullptr;
            cap = 0;
        }
        hipError_t e = hipMalloc(&p, bytes);
        if (e == hipSuccess) cap = bytes;
        return e;
    }
    template <class T> T* as() const { return static_cast<T*>(p); }
};

struct HostPinned {
    void* p = nullptr;
    size_t cap = 0;
    HostPinned() = default;
    HostPinned(const HostPinned&) = delete;
    HostPinned& operator=(const HostPinned&) = delete;
    ~HostPinned() {
        if (p) (void)hipHostFree(p);
    }
    hipError_t reserve(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) {
            (void)hipHostFree(p);
            p = nullptr;
            cap = 0;
        }
        hipError_t e = hipHostMalloc(&p, bytes, hipHostMallocDefault);
        if (e == hipSuccess) cap = bytes;
        return e;
    }
};

inline int units_for(int dim, int enc) { return enc == ENC_FLOAT32 ? (dim + 3) / 4 : (dim + 15) / 16; }

}  // namespace osk

struct osk_seg {
    int device = 0;
    int64_t n_rows = 0;
    int dim = 0, enc = 0, sim = 0, max_doc = 0;
    int units = 0, cfg = 0;
    void* d_rows = nullptr;
    float* d_xnorm_f = nullptr;
    int32_t* d_xnorm_i = nullptr;
    int32_t* d_ord_to_doc = nullptr;
    // batched MFMA path (built by osk_seg_warm or on first batched search): bf16 hi/lo copy in MFMA
    // fragment order, |x|² per row (device lane order) and max |x|² of the segment
    void* d_split = nullptr;
    int split_KS = 0;
    unsigned* d_maxnorm2 = nullptr;
    float* d_xsqrt = nullptr;          // |x| per row (MFMA path)
    float h_maxnorm2 = 0.0f;
    // certified int8 prefilter (built at staging for float32 segments): int8 rows + per-row bound terms
    void* d_q8 = nullptr;
    float4* d_q8aux = nullptr;
    void* d_q8t = nullptr;    // the int8 rows in sq8_mfma's tiled layout (osk_seg_warm / first batched prefilter)
    void* d_q8w = nullptr;        // sq8_wide's copy: codes with one scale per 16-row group, tiled (launch_sq8w_build)
    float4* d_q8auxt = nullptr;   // ...and its bound terms per 16-row group (built with d_q8t)
    void* d_q6 = nullptr;     // the 6-bit tier (dims with sq6_supported, tune sq6 on at staging): tiled codes,
    float4* d_q6aux = nullptr;   // built with the int8 copy; freed when the segment's calibration turns it off
    // The 6-bit tier's calibration, per segment: every view over the segment (a searcher's view, its
    // leased replicas, the next refresh's view) shares it.  Probe calls count, per segment, the rows they
    // re-bound from the int8 copy (read back asynchronously, osk_api.hip fold_probe); after kSq6Probes
    // probes the tier stays on, or turns off (above sq6_probe_pct % of the rows) and its copy is freed.
    std::atomic<int> sq6_state{0};     // 0 probing, 1 on, 2 off
    int sq6_probes = 0;                // (guarded by mu)
    int64_t sq6_probe_rows = 0, sq6_probe_rebound = 0;
    int units8 = 0;
    std::mutex mu;
    std::atomic<int> refs{1};          // the reader's reference + one per view that groups the segment
    osk_view* self_view = nullptr;     // single-segment view behind osk_seg_search (holds no reference)
    ~osk_seg();
    int64_t hbm_bytes() const;         // every device allocation the segment owns
};

struct osk_view {
    int device = 0, dim = 0, enc = 0, sim = 0, units = 0, cfg = 0;
    std::vector<osk_seg*> segs;
    bool holds_refs = true;            // false for a segment's own self_view
    std::vector<int32_t> seg_shard, seg_doc_base;
    int n_shards = 0;
    std::vector<int32_t> shard_index;
    std::vector<int32_t> shard_tile_begin;
    int n_tiles = 0;
    osk::DevBuf d_segs, d_tiles, d_shard_tile_begin, d_shard_index, d_tile_coff, d_tile_order;
    // workspace
    osk::DevBuf ws_cand, ws_q, ws_qnorm, ws_qin, ws_keys, ws_counts, ws_accept_ptrs, ws_accept,
        ws_out, ws_visited;
    osk::HostPinned h_stage;
    osk::HostPinned h_accept_tab;     // osk_view_search's accept pointer table (source of an async copy)
    // batched MFMA path
    bool mfma_ready = false;
    int n_munits = 0;
    int mfma_KS = 0;
    double mfma_c = 0.0;
    osk::DevBuf d_munits, d_seg_split, d_seg_xsqrt, d_seg_vrow, d_shard_unit_begin, d_shard_maxnorm2;
    osk::DevBuf ws_qsplit, ws_cand_a, ws_akeys, ws_acounts, ws_pkeys, ws_pcounts, ws_flags, ws_fbq, ws_fbkeys,
        ws_fbcounts;
    osk::HostPinned h_flags;
    int64_t mfma_calls = 0, mfma_fallback_queries = 0;
    osk::DevBuf d_mfma_full;               // [1] tiles whose candidate epilogue took the staging path
    // certified int8 prefilter
    bool sq8_ready = false;
    int units8 = 0;
    float sq8_gam = 0.f, sq8_g2 = 0.f, sq8_cos_slack = 0.f;
    osk::DevBuf d_sq8_rows, d_sq8_aux, d_counters;   // counters: SettleParams::counters
    osk::DevBuf d_sq8_rows_t;                         // per segment: tiled int8 copy (sq8_mfma)
    osk::DevBuf d_sq8_rows_w;                         // per segment: the wide kernel's group-scaled copy
    osk::DevBuf d_sq8_auxt, d_shard_quarter_begin;    // per segment: its tiled bound terms (sq8_wide); 4·shard_tile_begin
    osk::DevBuf d_quarter_bm;                         // per (wide tile, quarter): its rows' bound-term maxima
    osk::DevBuf d_wqtable;                            // per quarter in tile order: the wide kernels' descriptor
    // sq8_wide's own tiles (ensure_sq8w: quarters of ≈ R / (2·CUs) rows), their shard ranges and dispatch order
    osk::DevBuf d_wtiles, d_wtile_order, d_wshard_tile_begin;
    std::vector<int32_t> wshard_tile_begin;
    int n_wtiles = 0;
    bool sq8t_ready = false;   // sq8_mfma's tiled copy pointers (ensure_sq8t)
    bool sq8w_ready = false;   // the wide kernel's copies, pointers and tile table (ensure_sq8w)
    osk::DevBuf d_sq6_rows, d_sq6_aux;                // per segment: the 6-bit tier (every segment has one or
    bool sq6_ready = false;                           // the view does not use it)
    int64_t sq6_calls = 0;
    osk::DevBuf ws_q6, ws_qc6, ws_floor;              // its query (nibble split, bound terms), floor buckets,
    osk::DevBuf ws_cand6, ws_cnt6;                    // the streaming pass's candidates per list {row, 6-bit test}
    // the tier's calibration (per segment, osk_seg::sq6_state): a probe call of this view counts its int8
    // re-bounds per segment into d_seg_rebound, copies them to h_seg_rebound on its stream and records
    // ev_probe; a later call folds them into the segments once the event has completed — nothing waits
    osk::DevBuf d_seg_rebound;
    osk::HostPinned h_seg_rebound;
    hipEvent_t ev_probe = nullptr;
    bool probe_pending = false;
    osk::DevBuf ws_q8, ws_qc, ws_sq8cand, ws_sq8lb, ws_lbmax, ws_trace;
    // settle slices: kSliceLists wave lists each, never spanning shards (an empty shard gets one
    // empty slice so that its result is still written)
    int n_slices = 0;
    osk::DevBuf d_slices, d_shard_slice_begin, ws_part;
    osk::DevBuf ws_pilot, ws_thr, ws_thr_counts;   // int8 MFMA prefilter: pilot keys, per-(query, shard) floors
    osk::DevBuf ws_wfloor;                          // sq8_wide: the two passes' floors [2][kWideQ][S]
    int64_t sq8_calls = 0, sq8w_calls = 0;
    int n_cus = 0;                         // the device's CUs (cached; the wide kernel's persistent grid)   // prefiltered searches; those whose batch took sq8_wide
    // filter pushdown by compaction (osk_filter.hip): gather tiles over the compacted accepted ordinals
    // (one round of the chip, split over segments by rows), their settle slices, per-segment tile ranges
    // the select path (osk_select.hip, any k): per-row records of one query, radix state, candidates
    osk::DevBuf ws_sel_lb, ws_sel_ub, ws_sel_keys, ws_sel_state, ws_sel_hist, ws_sel_cand, ws_sel_cand2, ws_sel_cnt;
    int64_t sel_calls = 0;
    bool gather_ready = false;
    int n_gtiles = 0, n_gslices = 0;
    osk::DevBuf d_gtiles, d_gslices, d_gshard_slice_begin, d_seg_tiles;
    osk::DevBuf ws_tcnt, ws_scnt, ws_comp;
    // multi-GPU exchange (osk_comm.hip): this rank's block (lists padded to the call's shards per rank,
    // header, shard indices), the gathered blocks of every rank, the host entry's reduce outputs
    osk::DevBuf ws_xkeys, ws_xgath, ws_xout, ws_xspr;
    std::mutex mu;
    // scan-kernel timing (osk_view_profile): a ring of (start, stop) event pairs, one per search call,
    // folded into scan_ms when a slot is reused (kEvRing calls later: long complete, no host wait) or
    // when the total is read — timing never blocks the host inside the timed loop
    static constexpr int kEvRing = 64;
    bool profile = false;            // the current call stamps its scan launches (osk_view_profile)
    int profile_every = 0;           // osk_view_profile(enable): 0 off, N = every N-th call is sampled
    uint64_t profile_tick = 0;
    hipEvent_t ev_start[kEvRing] = {}, ev_stop[kEvRing] = {};
    bool ev_pending[kEvRing] = {};
    int64_t ev_next = 0;                  // calls started since enabling
    hipEvent_t ev0 = nullptr, ev1 = nullptr;   // the current call's pair
    hipEvent_t ev_call[2] = {};                 // host entries' per-call device time (tune call_timing)
    double scan_ms = 0.0;
    int64_t scan_calls = 0;
    const uint64_t* h_accept_ptr = nullptr;   // source of osk_seg_search's one-pointer accept table copy
    // cross-stream ordering of the workspace: the stream of the previous search, and an event recorded
    // on it when a search arrives on another stream (order_after_last)
    hipStream_t last_stream = nullptr;
    hipEvent_t xs_event = nullptr;
    // Host entries (osk_view_search, osk_seg_search) are synchronous calls from the search thread
    // pools.  Each concurrent call leases a workspace slot — slot 0 is this view, slot i > 0 a replica
    // view over the same segments (own workspace) — and the slot's own stream, so concurrent searches
    // of one shard set run concurrently on the device instead of queueing on one workspace.
    static constexpr int kMaxLeases = 8;
    std::mutex lease_mu;
    std::condition_variable lease_cv;
    std::vector<osk_view*> replicas;          // slots 1.. (created on demand)
    std::vector<hipStream_t> lease_streams;   // one per slot
    std::vector<char> lease_busy;             // per slot
    // opportunistic batching of concurrent host calls (osk_api.hip batched_call)
    struct Batcher {
        std::mutex mu;
        std::condition_variable cv;
        std::deque<void*> queue;              // waiting requests (BatchReq*)
        int leaders = 0;                      // batches in flight
        int64_t batches = 0, requests = 0;
    } batcher;
    ~osk_view();
};

namespace osk {
// Drop one reference of a segment (deletes it at zero).
void seg_unref(osk_seg* s);
// Order this call's use of the view's workspace after the previous call's (another stream).
int32_t order_after_last(osk_view* v, hipStream_t st);
// A leased workspace slot of a view (host entries): `v` is the view or one of its replicas, `st` the
// slot's stream.  Released (and a waiting caller woken) when the lease goes out of scope.
struct ViewLease {
    osk_view* root = nullptr;
    osk_view* v = nullptr;
    hipStream_t st = nullptr;
    int slot = -1;
    ViewLease() = default;
    ViewLease(const ViewLease&) = delete;
    ViewLease& operator=(const ViewLease&) = delete;
    ~ViewLease();
};
int32_t lease_view(osk_view* root, ViewLease& out);
// Per-shard exact top-k on the device (caller holds v->mu; device current).
int32_t view_search_device(osk_view* v, const void* d_queries, int nq, int k, const uint64_t* const* d_accept,
                           uint64_t* d_shard_keys, int32_t* d_shard_counts, int64_t* d_visited, hipStream_t st);
}  // namespace osk
