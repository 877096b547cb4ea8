// osk_comm.hip — the multi-GPU exchange of libosknn: one index shard per GPU, ONE RCCL all-gather of
// every GPU's per-shard top-k lists over xGMI, and the coordinator reduce on the device.
//
// Reference semantics mirrored:
//   * shards are OpenSearch's partitioning (S/cluster/metadata/IndexMetadata.java:265-268); the
//     coordinator fans a query out to one copy of every shard (S/action/search/
//     AbstractSearchAsyncAction.java:262-268) whose loop index is the shardIndex
//     (S/cluster/routing/GroupShardsIterator.java:59-62);
//   * the per-shard results are reduced by SearchPhaseController.mergeTopDocs → [L] TopDocs.merge
//     (S/action/search/SearchPhaseController.java:224-246, setShardIndex :248-253): score desc, then
//     shardIndex asc, then doc asc, cut to from+size; TopDocsStats (:839-901) for total hits and max
//     score.
// Design: each GPU scans its shards in one launch and writes per-shard lists of 8-byte
// hit keys [nq][shards_per_rank][k] (key 0 = empty); one ncclAllGather moves them to every GPU
// (8·k·nq bytes per shard: latency-bound, µs next to a ms scan); merge_coord then runs straight over
// the gathered rank-major image.  A list's hit count is its number of non-zero keys, so counts are not
// exchanged.  Each rank's block also carries its shard indices and a call header (sequence number,
// batch shape, query fingerprint) that the reduce checks across ranks, so ranks that issued different
// calls get an error instead of a merge of unrelated lists (see "the exchange block" below).
//
// RCCL is loaded at run time (dlopen of librccl.so.1, preferring a copy the process already loaded,
// e.g. PyTorch's), so the library itself has no link-time dependency on it and every other entry point
// works where RCCL is absent; the communicator entry points then fail with OSK_ERR_UNSUPPORTED.
#include <dlfcn.h>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <thread>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "osk_objects.h"

using namespace osk;

struct osk_comm {
    uint64_t id = 0;                     // process-unique, never reused (views cache per-comm state by it)
    int rank = 0, world = 1;             // rank of local device 0, communicator size
    std::vector<int> devices;            // local devices: 1 (one process per GPU) or all (one process)
    std::vector<ncclComm_t> comms;       // one per local device
    // one exchange stream per local device: every collective of the communicator is issued on it, in
    // call order, whatever stream (search thread) the call arrived on — RCCL needs one issue order per
    // communicator, and a search's scan on its own stream overlaps the previous search's exchange
    std::vector<hipStream_t> xstreams;
    // per local device: "inputs ready" (caller stream → exchange stream) and "outputs ready" (back);
    // reused by every call: calls are serialised by `mu`, and a stream wait binds the record before it
    std::vector<hipEvent_t> ev_in, ev_out;
    std::mutex mu;                       // one collective sequence at a time
    uint64_t seq = 0;                    // calls issued (the exchange header's sequence number)
    // [mismatch flag, rank 0's sequence number, first mismatching rank, its sequence number], written by
    // the reduce kernel (pinned host memory); a set flag makes the communicator refuse further calls
    osk::HostPinned h_err;
    osk::HostPinned h_spr;               // the host entry's call agreement (agree_call)
    // the device entry's exchange limits (osk_comm_set_device_limits): its world > 1 block has this fixed size
    int dev_max_nq = 1, dev_max_k = 100, dev_max_spr = 8;
    void* lb = nullptr;                  // testing build: loopback transport instead of RCCL
    bool lb_local = false;               // testing build: init_all's local devices exchange by device copies
    void (*lb_free)(void*) = nullptr;
    ~osk_comm() {
        if (lb_free) lb_free(lb);
        for (size_t i = 0; i < devices.size(); ++i) {
            (void)hipSetDevice(devices[i]);
            if (i < xstreams.size() && xstreams[i]) (void)hipStreamDestroy(xstreams[i]);
            if (i < ev_in.size() && ev_in[i]) (void)hipEventDestroy(ev_in[i]);
            if (i < ev_out.size() && ev_out[i]) (void)hipEventDestroy(ev_out[i]);
        }
    }
};

namespace {

std::atomic<uint64_t> g_comm_ids{0};

struct Rccl {
    ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

std::once_flag g_rccl_once;
Rccl g_rccl;
bool g_rccl_ok = false;
std::string g_rccl_err;

void load_rccl() {
    // a copy already in the process first (RTLD_NOLOAD), then the system one
    void* h = nullptr;
    for (const char* name : {"librccl.so.1", "librccl.so"})
        if (!h) h = dlopen(name, RTLD_NOW | RTLD_LOCAL | RTLD_NOLOAD);
    for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
        if (!h) h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
    if (!h) {
        const char* e = dlerror();
        g_rccl_err = std::string("RCCL (librccl.so.1) could not be loaded: ") + (e ? e : "unknown error");
        return;
    }
    auto sym = [&](const char* n) { return dlsym(h, n); };
    g_rccl.GetUniqueId = reinterpret_cast<decltype(g_rccl.GetUniqueId)>(sym("ncclGetUniqueId"));
    g_rccl.CommInitRank = reinterpret_cast<decltype(g_rccl.CommInitRank)>(sym("ncclCommInitRank"));
    g_rccl.CommInitAll = reinterpret_cast<decltype(g_rccl.CommInitAll)>(sym("ncclCommInitAll"));
    g_rccl.CommDestroy = reinterpret_cast<decltype(g_rccl.CommDestroy)>(sym("ncclCommDestroy"));
    g_rccl.AllGather = reinterpret_cast<decltype(g_rccl.AllGather)>(sym("ncclAllGather"));
    g_rccl.GroupStart = reinterpret_cast<decltype(g_rccl.GroupStart)>(sym("ncclGroupStart"));
    g_rccl.GroupEnd = reinterpret_cast<decltype(g_rccl.GroupEnd)>(sym("ncclGroupEnd"));
    g_rccl.GetErrorString = reinterpret_cast<decltype(g_rccl.GetErrorString)>(sym("ncclGetErrorString"));
    if (!g_rccl.GetUniqueId || !g_rccl.CommInitRank || !g_rccl.CommInitAll || !g_rccl.CommDestroy ||
        !g_rccl.AllGather || !g_rccl.GroupStart || !g_rccl.GroupEnd || !g_rccl.GetErrorString) {
        g_rccl_err = "librccl is missing an nccl* entry point";
        return;
    }
    g_rccl_ok = true;
}

const Rccl* rccl() {
    std::call_once(g_rccl_once, load_rccl);
    if (!g_rccl_ok) {
        set_error(g_rccl_err);
        return nullptr;
    }
    return &g_rccl;
}

#define OSK_NCCL(call)                                                                         \
    do {                                                                                       \
        ncclResult_t r_ = (call);                                                              \
        if (r_ != ncclSuccess) {                                                               \
            set_error(std::string(#call) + ": " + g_rccl.GetErrorString(r_));                  \
            return OSK_ERR_DEVICE;                                                             \
        }                                                                                      \
    } while (0)

int32_t make_xstreams(osk_comm* c) {
    const size_t n = c->devices.size();
    c->xstreams.assign(n, nullptr);
    c->ev_in.assign(n, nullptr);
    c->ev_out.assign(n, nullptr);
    for (size_t i = 0; i < n; ++i) {
        OSK_HIP(hipSetDevice(c->devices[i]));
        OSK_HIP(hipStreamCreateWithFlags(&c->xstreams[i], hipStreamNonBlocking));
        OSK_HIP(hipEventCreateWithFlags(&c->ev_in[i], hipEventDisableTiming));
        OSK_HIP(hipEventCreateWithFlags(&c->ev_out[i], hipEventDisableTiming));
    }
    OSK_HIP(c->h_err.reserve(4 * sizeof(int64_t)));
    std::memset(c->h_err.p, 0, 4 * sizeof(int64_t));
    return OSK_OK;
}

// Work enqueued on `st` so far → before the next operation on local device i's exchange stream.
hipError_t enter_xstream(osk_comm* c, size_t i, hipStream_t st) {
    hipError_t e = hipEventRecord(c->ev_in[i], st);
    return e != hipSuccess ? e : hipStreamWaitEvent(c->xstreams[i], c->ev_in[i], 0);
}

// Everything enqueued on the exchange stream so far → before the next operation on `st`.
hipError_t leave_xstream(osk_comm* c, size_t i, hipStream_t st) {
    hipError_t e = hipEventRecord(c->ev_out[i], c->xstreams[i]);
    return e != hipSuccess ? e : hipStreamWaitEvent(st, c->ev_out[i], 0);
}

// The per-shard lists of one view, padded to `spr` shards per rank: ws_xkeys [nq][spr][k].
// ws_keys [nq][n_shards][k] → ws_xkeys [nq][spr][k], the pad slots zero (empty lists).
int32_t pad_lists(osk_view* v, int nq, int k, int spr, hipStream_t st) {
    uint64_t* xk = v->ws_xkeys.as<uint64_t>();
    OSK_HIP(hipMemsetAsync(xk, 0, sizeof(uint64_t) * nq * spr * k, st));
    OSK_HIP(hipMemcpy2DAsync(xk, sizeof(uint64_t) * spr * k, v->ws_keys.p, sizeof(uint64_t) * v->n_shards * k,
                             sizeof(uint64_t) * v->n_shards * k, nq, hipMemcpyDeviceToDevice, st));
    return OSK_OK;
}

int32_t search_padded(osk_view* v, const void* d_queries, int nq, int k, const uint64_t* const* d_accept, int spr,
                      hipStream_t st) {
    const size_t per = (size_t)nq * spr * k;
    OSK_HIP(v->ws_xkeys.reserve(sizeof(uint64_t) * per));
    OSK_HIP(v->ws_counts.reserve(sizeof(int32_t) * (size_t)nq * v->n_shards));
    uint64_t* xk = v->ws_xkeys.as<uint64_t>();
    if (v->n_shards == spr)
        return view_search_device(v, d_queries, nq, k, d_accept, xk, v->ws_counts.as<int32_t>(), nullptr, st);
    OSK_HIP(v->ws_keys.reserve(sizeof(uint64_t) * (size_t)nq * v->n_shards * k));
    int32_t rc = view_search_device(v, d_queries, nq, k, d_accept, v->ws_keys.as<uint64_t>(),
                                    v->ws_counts.as<int32_t>(), nullptr, st);
    if (rc) return rc;
    return pad_lists(v, nq, k, spr, st);
}

// ---- the exchange block ------------------------------------------------------------------------
// Rank block (u64 words): [keys nq·spr·k][header kXHdrWords][shard indices spr int32, padded to words].
// Every call gathers whole blocks, so each call carries its own shardIndex (no cached exchange state a
// rank could disagree about) and a header the reduce compares across ranks (osk_device.h
// xchg_header_check): call sequence number, batch, k, from/size, shards per rank, dim/encoding and a
// fingerprint of the query bytes.  Ranks that issued different calls get count −1 on every query and
// a sticky error on the communicator instead of merging keys of different queries.
struct Block {
    size_t keys, words;
};
Block block_of(int nq, int k, int spr) {
    const size_t keys = (size_t)nq * spr * k;
    return {keys, keys + kXHdrWords + (size_t)(spr + 1) / 2};
}

// ("OSKX" block format 1: kXMagic, osk_internal.h; kXRefused marks a refusing rank's block)

// Header words of this call (w[5], the query fingerprint, is computed on the device).
void header_words(uint64_t (&w)[kXHdrWords], uint64_t seq, int nq, int k, int from, int size, int spr, int dim,
                  int enc, int world) {
    w[0] = kXMagic;
    w[1] = seq;
    w[2] = (uint32_t)nq | ((uint64_t)(uint32_t)k << 32);
    w[3] = (uint32_t)from | ((uint64_t)(uint32_t)size << 32);
    w[4] = (uint32_t)spr | ((uint64_t)(uint32_t)(dim | enc << 16) << 32);
    w[5] = 0;
    w[6] = (uint64_t)world;
    w[7] = 0;
}

int32_t poisoned(const osk_comm* c) {
    const int64_t* e = static_cast<const int64_t*>(c->h_err.p);
    if (!e || !e[0]) return OSK_OK;
    set_error("communicator poisoned: the ranks issued different calls (rank 0 at call " + std::to_string(e[1]) +
              ", rank " + std::to_string(e[2]) + " at call " + std::to_string(e[3]) +
              "); every rank must issue the same searches in the same order — release and re-create it");
    return OSK_ERR_INVALID;
}

#ifdef OSK_TESTING
// ---- loopback transport (testing build only) -----------------------------------------------------
// Lets one GPU host several ranks (RCCL refuses two ranks on one device), so the world > 1 code of
// this file runs on a one-GPU box: the all-gather goes through a POSIX shared-memory segment.  Per
// call g every rank copies its block into slot [g & 1][rank], publishes gen[rank] = g, waits for every
// rank's gen ≥ g, copies all slots into its receive buffer and publishes read[rank] = g; a slot is
// rewritten (call g + 2) only once every rank has read call g.  A peer that does not arrive within
// kLoopbackTimeoutS is an error, not a hang.
struct Loopback {
    static constexpr int kMaxWorld = 64;
    static constexpr double kTimeoutS = 120.0;
    struct Ctrl {
        std::atomic<int64_t> joined;
        std::atomic<int64_t> gen[kMaxWorld];
        std::atomic<int64_t> read[kMaxWorld];
        std::atomic<int64_t> bytes[2][kMaxWorld];
    };
    int rank = 0, world = 1;
    size_t slot_bytes = 0, map_bytes = 0;
    void* base = nullptr;
    int fd = -1;
    std::string name;
    int64_t gen = 0;
    Ctrl* ctrl() const { return static_cast<Ctrl*>(base); }
    char* slot(int par, int r) const {
        return static_cast<char*>(base) + 4096 + ((size_t)par * world + r) * slot_bytes;
    }
    ~Loopback() {
        if (base) munmap(base, map_bytes);
        if (fd >= 0) close(fd);
        if (rank == 0 && !name.empty()) shm_unlink(name.c_str());
    }
    // every rank's counter ≥ want (false: timed out)
    bool wait_all(std::atomic<int64_t>* a, int64_t want) const {
        const auto t0 = std::chrono::steady_clock::now();
        for (int r = 0; r < world; ++r)
            while (a[r].load(std::memory_order_acquire) < want) {
                if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > kTimeoutS)
                    return false;
                std::this_thread::sleep_for(std::chrono::microseconds(20));
            }
        return true;
    }
};

int32_t lb_allgather(Loopback* L, const void* d_send, void* d_recv, size_t bytes, hipStream_t st) {
    OSK_REQUIRE(bytes <= L->slot_bytes, "loopback all-gather: the block is larger than the slot");
    Loopback::Ctrl* c = L->ctrl();
    const int64_t g = ++L->gen;
    const int par = (int)(g & 1);
    if (!L->wait_all(c->read, g - 2)) {   // slot [par][rank] is free once every rank has read call g − 2
        set_error("loopback all-gather: a peer never finished reading call " + std::to_string(g - 2));
        return OSK_ERR_DEVICE;
    }
    OSK_HIP(hipMemcpyAsync(L->slot(par, L->rank), d_send, bytes, hipMemcpyDeviceToHost, st));
    OSK_HIP(hipStreamSynchronize(st));
    c->bytes[par][L->rank].store((int64_t)bytes, std::memory_order_relaxed);
    c->gen[L->rank].store(g, std::memory_order_release);
    if (!L->wait_all(c->gen, g)) {
        set_error("loopback all-gather: a peer never issued call " + std::to_string(g));
        return OSK_ERR_DEVICE;
    }
    bool same = true;
    for (int r = 0; r < L->world; ++r) same &= c->bytes[par][r].load(std::memory_order_relaxed) == (int64_t)bytes;
    for (int r = 0; same && r < L->world; ++r)
        OSK_HIP(hipMemcpyAsync(static_cast<char*>(d_recv) + (size_t)r * bytes, L->slot(par, r), bytes,
                               hipMemcpyHostToDevice, st));
    OSK_HIP(hipStreamSynchronize(st));
    c->read[L->rank].store(g, std::memory_order_release);
    OSK_REQUIRE(same, "loopback all-gather: the ranks passed blocks of different sizes");
    return OSK_OK;
}

// Testing build: the grouped all-gather of one process's n local devices (osk_comm_init_all) as device
// copies, so the multi-device code of the host entry runs with every local "device" mapped to one GPU
// (RCCL refuses two ranks on one device).  Local device i = rank i; send r → slot r of every receive
// buffer.  The host waits for every send (its exchange stream drained) before copying: the transport
// stands in for the collective, its latency is not the product's.
int32_t local_allgather(osk_comm* c, const void* const* sends, void* const* recvs, size_t bytes) {
    const size_t n = c->devices.size();
    OSK_REQUIRE(n == (size_t)c->world, "local all-gather: one rank per local device");
    // Ordering: every caller of gather_blocks first makes each exchange stream wait on the stream that
    // produced its rank's send block (enter_xstream in osk_shards_search_merge_device / osk_shards_search_merge),
    // so draining the exchange streams here also drains the send blocks' producers — the same event chain
    // the RCCL all-gather relies on.  A caller that skipped enter_xstream would fail both transports alike.
    for (size_t i = 0; i < n; ++i) {
        OSK_HIP(hipSetDevice(c->devices[i]));
        OSK_HIP(hipStreamSynchronize(c->xstreams[i]));
    }
    for (size_t i = 0; i < n; ++i) {
        OSK_HIP(hipSetDevice(c->devices[i]));
        for (size_t r = 0; r < n; ++r)
            OSK_HIP(hipMemcpyAsync(static_cast<char*>(recvs[i]) + r * bytes, sends[r], bytes, hipMemcpyDefault,
                                   c->xstreams[i]));
    }
    return OSK_OK;
}
#endif

// One all-gather of every local view's block (ws_xkeys, `words` u64) into its ws_xgath, on the
// communicator's exchange streams (grouped over local devices).
int32_t gather_blocks(osk_comm* c, osk_view* const* views, size_t words, const hipStream_t* sts) {
    for (size_t i = 0; i < c->devices.size(); ++i) {
        OSK_HIP(hipSetDevice(views[i]->device));
        OSK_HIP(views[i]->ws_xgath.reserve(sizeof(uint64_t) * words * c->world));
    }
#ifdef OSK_TESTING
    if (c->lb) return lb_allgather(static_cast<Loopback*>(c->lb), views[0]->ws_xkeys.p, views[0]->ws_xgath.p,
                                   words * 8, sts[0]);
    if (c->lb_local) {
        std::vector<const void*> sends(c->devices.size());
        std::vector<void*> recvs(c->devices.size());
        for (size_t i = 0; i < c->devices.size(); ++i) {
            sends[i] = views[i]->ws_xkeys.p;
            recvs[i] = views[i]->ws_xgath.p;
        }
        return local_allgather(c, sends.data(), recvs.data(), words * 8);
    }
#endif
    OSK_NCCL(g_rccl.GroupStart());
    for (size_t i = 0; i < c->devices.size(); ++i)
        OSK_NCCL(g_rccl.AllGather(views[i]->ws_xkeys.p, views[i]->ws_xgath.p, words, ncclUint64, c->comms[i], sts[i]));
    OSK_NCCL(g_rccl.GroupEnd());
    return OSK_OK;
}

// This rank's block of one view: the trailer (header + shard indices) and the per-shard lists padded to
// spr shards.
int32_t fill_block(osk_view* v, const void* d_queries, int nq, int k, const uint64_t* const* d_accept, int spr,
                   const uint64_t (&hw)[kXHdrWords], hipStream_t st, const Block* cap = nullptr) {
    // (cap: the device entry's fixed block — the call's lists at its start, the header at cap->keys)
    const Block B = cap ? *cap : block_of(nq, k, spr);
    OSK_HIP(v->ws_xkeys.reserve(sizeof(uint64_t) * std::max(B.words, (size_t)nq * spr * k)));
    const int64_t qbytes = (int64_t)nq * v->dim * (v->enc == ENC_FLOAT32 ? 4 : 1);
    OSK_HIP(launch_xhdr_fill(v->ws_xkeys.as<uint64_t>() + B.keys, hw, d_queries, qbytes,
                             v->d_shard_index.as<int32_t>(), v->n_shards, spr, st));
    return search_padded(v, d_queries, nq, k, d_accept, spr, st);
}

// The device entry's fixed block at world > 1: the limits' keys region, the header, the limits' shard slots.
Block fixed_block_of(const osk_comm* c) {
    const size_t keys = (size_t)c->dev_max_nq * c->dev_max_spr * c->dev_max_k;
    return {keys, keys + kXHdrWords + (size_t)(c->dev_max_spr + 1) / 2};
}

// The reduce's view of a gathered (or, world 1, local) image of blocks.
XLayout image_layout(const osk_comm* c, const uint64_t* image, const Block& B, const int32_t** shard_index) {
    XLayout x;
    x.rank_words = B.words;
    x.si_stride = (int)(2 * B.words);
    x.hdr = image + B.keys;
    x.err = static_cast<int64_t*>(c->h_err.p);
    *shard_index = reinterpret_cast<const int32_t*>(image + B.keys + kXHdrWords);
    return x;
}

// The host entry's call agreement, before any variable-size collective: every rank gathers a fixed-size
// call header (sequence number, batch, k, from/size, dim/encoding, world; and its view's shard count) on
// the exchange streams and the host compares them (the scans already run).  RCCL requires every rank to
// pass the same count to ncclAllGather, and the block size depends on the batch, k and the shards per
// rank, so a rank that issued another call must be caught HERE — a block gather with different counts is
// undefined behaviour (a hang or garbage), never a header mismatch.  Every rank sees the same gathered
// headers, so every rank refuses together (and poisons its communicator) or proceeds together.  Shards
// per rank = the largest view of any rank (ranks may hold different numbers of shards: 8 over 3 GPUs),
// agreed on every call rather than cached (a cache would let ranks disagree on whether to exchange).
constexpr int kCallWords = 8;
int32_t agree_call(osk_comm* c, osk_view* const* views, int nq, int k, int from, int size, int* spr) {
    const size_t nl = c->devices.size(), W = (size_t)c->world;
    OSK_HIP(c->h_spr.reserve(sizeof(int64_t) * kCallWords * (nl + W)));
    int64_t* h = static_cast<int64_t*>(c->h_spr.p);   // [nl][kCallWords] send values, then [W][kCallWords] received
    for (size_t i = 0; i < nl; ++i) {
        osk_view* v = views[i];
        int64_t* w = h + i * kCallWords;
        w[0] = (int64_t)kXMagic;
        w[1] = (int64_t)(c->seq + 1);
        w[2] = (int64_t)((uint32_t)nq | ((uint64_t)(uint32_t)k << 32));
        w[3] = (int64_t)((uint32_t)from | ((uint64_t)(uint32_t)size << 32));
        w[4] = (int64_t)(v->dim | v->enc << 16);
        w[5] = c->world;
        w[6] = v->n_shards;
        w[7] = 0;
        OSK_HIP(hipSetDevice(v->device));
        OSK_HIP(v->ws_xspr.reserve(sizeof(int64_t) * kCallWords * (W + 1)));
        OSK_HIP(hipMemcpyAsync(v->ws_xspr.as<int64_t>() + W * kCallWords, w, 8 * kCallWords, hipMemcpyHostToDevice,
                               c->xstreams[i]));
    }
#ifdef OSK_TESTING
    if (c->lb) {
        int32_t rc = lb_allgather(static_cast<Loopback*>(c->lb), views[0]->ws_xspr.as<int64_t>() + W * kCallWords,
                                  views[0]->ws_xspr.p, 8 * kCallWords, c->xstreams[0]);
        if (rc) return rc;
    } else if (c->lb_local) {
        std::vector<const void*> sends(nl);
        std::vector<void*> recvs(nl);
        for (size_t i = 0; i < nl; ++i) {
            sends[i] = views[i]->ws_xspr.as<int64_t>() + W * kCallWords;
            recvs[i] = views[i]->ws_xspr.p;
        }
        int32_t rc = local_allgather(c, sends.data(), recvs.data(), 8 * kCallWords);
        if (rc) return rc;
    } else
#endif
    {
        OSK_NCCL(g_rccl.GroupStart());
        for (size_t i = 0; i < nl; ++i)
            OSK_NCCL(g_rccl.AllGather(views[i]->ws_xspr.as<int64_t>() + W * kCallWords, views[i]->ws_xspr.p,
                                      kCallWords, ncclInt64, c->comms[i], c->xstreams[i]));
        OSK_NCCL(g_rccl.GroupEnd());
    }
    int64_t* recv = h + nl * kCallWords;
    OSK_HIP(hipSetDevice(views[0]->device));
    OSK_HIP(hipMemcpyAsync(recv, views[0]->ws_xspr.p, 8 * kCallWords * W, hipMemcpyDeviceToHost, c->xstreams[0]));
    for (size_t i = 0; i < nl; ++i) {
        OSK_HIP(hipSetDevice(views[i]->device));
        OSK_HIP(hipStreamSynchronize(c->xstreams[i]));
    }
    int m = 1;
    for (size_t r = 0; r < W; ++r) {
        const int64_t* w = recv + r * kCallWords;
        for (int j = 0; j < 6; ++j)
            if (w[j] != recv[j]) {   // another call on rank r: refuse on every rank, before the block gather
                int64_t* e = static_cast<int64_t*>(c->h_err.p);
                e[1] = recv[1];
                e[2] = (int64_t)r;
                e[3] = w[1];
                e[0] = 1;
                return poisoned(c);
            }
        m = std::max<int>(m, (int)w[6]);
    }
    *spr = m;
    return OSK_OK;
}

int32_t check_merge_args(const osk_comm* c, int nq, int k, int from, int size, int spr) {
    OSK_REQUIRE(nq >= 1, "n_queries must be >= 1");
    OSK_REQUIRE(k >= 1 && k <= OSK_MAX_K, "k must be in [1, OSK_MAX_K]");
    OSK_REQUIRE(from >= 0 && size >= 1 && (int64_t)from + size <= 100000, "bad from/size");
    OSK_REQUIRE(spr >= 1, "shards_per_rank must be >= 1");
    return OSK_OK;
}

}  // namespace

extern "C" {

int32_t osk_comm_unique_id(uint8_t* id) {
    OSK_GUARD_BEGIN
    clear_error();
    OSK_REQUIRE(id != nullptr, "id is null");
    if (device_count_cached() <= 0) {   // RCCL needs a device even to make an id
        set_error("no HIP device visible (libosknn has no CPU fallback)");
        return OSK_ERR_NO_DEVICE;
    }
    const Rccl* R = rccl();
    if (!R) return OSK_ERR_UNSUPPORTED;
    ncclUniqueId u;
    OSK_NCCL(R->GetUniqueId(&u));
    static_assert(sizeof(u) == OSK_COMM_ID_BYTES, "ncclUniqueId size");
    std::memcpy(id, &u, sizeof(u));
    return OSK_OK;
    OSK_GUARD_END
}

int32_t osk_comm_init_rank(int32_t device, int32_t rank, int32_t world, const uint8_t* id, osk_comm** out) {
    OSK_GUARD_BEGIN
    clear_error();
    OSK_REQUIRE(out != nullptr && id != nullptr, "null argument");
    OSK_REQUIRE(world >= 1 && rank >= 0 && rank < world, "need 0 <= rank < world");
    int32_t rc = check_device(device);
    if (rc) return rc;
    const Rccl* R = rccl();
    if (!R) return OSK_ERR_UNSUPPORTED;
    auto c = std::make_unique<osk_comm>();
    c->id = ++g_comm_ids;
    c->rank = rank;
    c->world = world;
    c->devices = {device};
    c->comms.assign(1, nullptr);
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    OSK_NCCL(R->CommInitRank(&c->comms[0], world, u, rank));
    rc = make_xstreams(c.get());
    if (rc) {
        (void)R->CommDestroy(c->comms[0]);
        return rc;
    }
    *out = c.release();
    return OSK_OK;
    OSK_GUARD_END
}

int32_t osk_comm_init_all(const int32_t* devices, int32_t n, osk_comm** out) {
    OSK_GUARD_BEGIN
    clear_error();
    OSK_REQUIRE(out != nullptr && devices != nullptr && n >= 1, "null argument");
    for (int i = 0; i < n; ++i) {
        int32_t rc = check_device(devices[i]);
        if (rc) return rc;
        for (int j = 0; j < i; ++j) OSK_REQUIRE(devices[j] != devices[i], "duplicate device");
    }
    const Rccl* R = rccl();
    if (!R) return OSK_ERR_UNSUPPORTED;
    auto c = std::make_unique<osk_comm>();
    c->id = ++g_comm_ids;
    c->rank = 0;
    c->world = n;
    c->devices.assign(devices, devices + n);
    c->comms.assign(n, nullptr);
    OSK_NCCL(R->CommInitAll(c->comms.data(), n, devices));
    int32_t rc = make_xstreams(c.get());
    if (rc) {
        for (int i = 0; i < n; ++i) {
            (void)hipSetDevice(devices[i]);
            (void)R->CommDestroy(c->comms[i]);
        }
        return rc;
    }
    *out = c.release();
    return OSK_OK;
    OSK_GUARD_END
}

int32_t osk_comm_release(osk_comm* comm) {
    OSK_GUARD_BEGIN
    if (!comm) return OSK_OK;
    for (size_t i = 0; i < comm->comms.size(); ++i)
        if (comm->comms[i]) {
            (void)hipSetDevice(comm->devices[i]);
            (void)g_rccl.CommDestroy(comm->comms[i]);
        }
    delete comm;
    return OSK_OK;
    OSK_GUARD_END
}

int32_t osk_comm_info(const osk_comm* comm, int32_t* rank, int32_t* world, int32_t* n_local) {
    OSK_GUARD_BEGIN
    OSK_REQUIRE(comm != nullptr, "comm is null");
    if (rank) *rank = comm->rank;
    if (world) *world = comm->world;
    if (n_local) *n_local = (int32_t)comm->devices.size();
    return OSK_OK;
    OSK_GUARD_END
}

int32_t osk_comm_all_gather(osk_comm* comm, const void* d_send, void* d_recv, int64_t bytes, void* stream) {
    OSK_GUARD_BEGIN
    clear_error();
    OSK_REQUIRE(comm != nullptr && d_send && d_recv && bytes >= 0, "null argument");
    OSK_REQUIRE(comm->devices.size() == 1, "osk_comm_all_gather needs a one-device-per-process communicator");
    int32_t rc = check_device(comm->devices[0]);
    if (rc) return rc;
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : device_stream(comm->devices[0]);
    std::lock_guard<std::mutex> lk(comm->mu);
    OSK_HIP(enter_xstream(comm, 0, st));
#ifdef OSK_TESTING
    if (comm->lb) {
        rc = lb_allgather(static_cast<Loopback*>(comm->lb), d_send, d_recv, (size_t)bytes, comm->xstreams[0]);
        if (rc) return rc;
    } else
#endif
        OSK_NCCL(g_rccl.AllGather(d_send, d_recv, (size_t)bytes, ncclUint8, comm->comms[0], comm->xstreams[0]));
    OSK_HIP(leave_xstream(comm, 0, st));
    return OSK_OK;
    OSK_GUARD_END
}

int32_t osk_comm_status(const osk_comm* comm, int64_t* info) {
    OSK_GUARD_BEGIN
    clear_error();
    OSK_REQUIRE(comm != nullptr, "comm is null");
    const int64_t* e = static_cast<const int64_t*>(comm->h_err.p);
    if (info)
        for (int i = 0; i < 4; ++i) info[i] = e ? e[i] : 0;
    return poisoned(comm);
    OSK_GUARD_END
}

int32_t osk_comm_init_loopback(int32_t device, int32_t rank, int32_t world, const uint8_t* id, int64_t slot_bytes,
                               osk_comm** out) {
    OSK_GUARD_BEGIN
    clear_error();
#ifndef OSK_TESTING
    (void)device; (void)rank; (void)world; (void)id; (void)slot_bytes; (void)out;
    set_error("osk_comm_init_loopback exists only in the testing build (libosknn_testing.so)");
    return OSK_ERR_UNSUPPORTED;
#else
    OSK_REQUIRE(out != nullptr && id != nullptr, "null argument");
    OSK_REQUIRE(world >= 1 && world <= Loopback::kMaxWorld && rank >= 0 && rank < world, "need 0 <= rank < world <= 64");
    OSK_REQUIRE(slot_bytes >= 4096 && slot_bytes <= (int64_t)1 << 30, "slot_bytes must be in [4 KiB, 1 GiB]");
    const size_t n = strnlen(reinterpret_cast<const char*>(id), OSK_COMM_ID_BYTES);
    OSK_REQUIRE(n > 1 && n < OSK_COMM_ID_BYTES && id[0] == '/', "loopback id: a NUL-terminated name \"/...\"");
    int32_t rc = check_device(device);
    if (rc) return rc;
    auto L = std::make_unique<Loopback>();
    L->rank = rank;
    L->world = world;
    L->slot_bytes = ((size_t)slot_bytes + 4095) & ~(size_t)4095;
    L->map_bytes = 4096 + 2 * (size_t)world * L->slot_bytes;
    L->name.assign(reinterpret_cast<const char*>(id), n);
    static_assert(sizeof(Loopback::Ctrl) <= 4096, "loopback control block");
    L->fd = shm_open(L->name.c_str(), O_CREAT | O_RDWR, 0600);
    OSK_REQUIRE(L->fd >= 0, "loopback: shm_open failed: " + std::string(strerror(errno)));
    OSK_REQUIRE(ftruncate(L->fd, (off_t)L->map_bytes) == 0, "loopback: ftruncate failed");
    L->base = mmap(nullptr, L->map_bytes, PROT_READ | PROT_WRITE, MAP_SHARED, L->fd, 0);
    if (L->base == MAP_FAILED) {
        L->base = nullptr;
        set_error("loopback: mmap failed");
        return OSK_ERR_OOM;
    }
    // (a fresh segment is zero-filled; every rank joins before the first call)
    L->ctrl()->joined.fetch_add(1);
    const auto t0 = std::chrono::steady_clock::now();
    while (L->ctrl()->joined.load() < world) {
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > Loopback::kTimeoutS) {
            set_error("loopback: not every rank joined");
            return OSK_ERR_DEVICE;
        }
        std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
    auto c = std::make_unique<osk_comm>();
    c->id = ++g_comm_ids;
    c->rank = rank;
    c->world = world;
    c->devices = {device};
    c->comms.assign(1, nullptr);
    rc = make_xstreams(c.get());
    if (rc) return rc;
    c->lb = L.release();
    c->lb_free = [](void* p) { delete static_cast<Loopback*>(p); };
    *out = c.release();
    return OSK_OK;
#endif
    OSK_GUARD_END
}

int32_t osk_comm_init_all_loopback(const int32_t* devices, int32_t n, osk_comm** out) {
    OSK_GUARD_BEGIN
    clear_error();
#ifndef OSK_TESTING
    (void)devices; (void)n; (void)out;
    set_error("osk_comm_init_all_loopback exists only in the testing build (libosknn_testing.so)");
    return OSK_ERR_UNSUPPORTED;
#else
    OSK_REQUIRE(out != nullptr && devices != nullptr && n >= 1 && n <= 64, "null argument or n outside [1, 64]");
    for (int i = 0; i < n; ++i) {
        int32_t rc = check_device(devices[i]);
        if (rc) return rc;
    }
    auto c = std::make_unique<osk_comm>();
    c->id = ++g_comm_ids;
    c->rank = 0;
    c->world = n;
    c->devices.assign(devices, devices + n);   // (may repeat: local "devices" mapped to one GPU)
    c->comms.assign(n, nullptr);
    int32_t rc = make_xstreams(c.get());
    if (rc) return rc;
    c->lb_local = true;
    *out = c.release();
    return OSK_OK;
#endif
    OSK_GUARD_END
}

int32_t osk_shards_search_merge_device(osk_comm* comm, osk_view* view, const void* d_queries, int32_t n_queries,
                                       int32_t k, const uint64_t* const* d_accept, int32_t shards_per_rank,
                                       int32_t from, int32_t size, float* d_scores, int32_t* d_docs,
                                       int32_t* d_shard_out, int32_t* d_count, int64_t* d_total_hits,
                                       float* d_max_score, void* stream) {
    OSK_GUARD_BEGIN
    clear_error();
    OSK_REQUIRE(comm != nullptr && view != nullptr && d_queries != nullptr, "null argument");
    OSK_REQUIRE(d_scores && d_docs && d_shard_out && d_count && d_total_hits && d_max_score, "null output");
    OSK_REQUIRE(comm->devices.size() == 1, "the device entry serves one-device-per-process communicators");
    OSK_REQUIRE(view->device == comm->devices[0], "the view is not on the communicator's device");
    // Argument errors of this rank alone (its shard count, batch, k, from/size).  At world 1 they return at
    // once.  At world > 1 the other ranks are about to enter the all-gather, so this rank must still issue
    // it: it sends the refusal header below (every rank's reduce then reports count −1 and the communicator
    // is poisoned), skips its own reduce (its output buffers may not fit the shape it was given) and returns
    // OSK_ERR_INVALID with the message.
    std::string local_err;
    if (view->n_shards > shards_per_rank) {
        local_err = "the view holds more shards than shards_per_rank";
    } else if (check_merge_args(comm, n_queries, k, from, size, shards_per_rank) != OSK_OK) {
        local_err = osk_last_error();
    }
    if (!local_err.empty() && comm->world == 1) {
        set_error(local_err);
        return OSK_ERR_INVALID;
    }
    int32_t rc = check_device(view->device);
    if (rc) return rc;
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : device_stream(view->device);
    // No refusal on the poison flag here: the previous call's reduce writes it asynchronously, so a rank
    // whose reduce had finished would refuse while a rank whose reduce had not would enter the all-gather
    // and wait forever.  Every call issues its collective; a poisoned communicator's reduce reports
    // count −1 on the device instead (xchg_header_check reads the sticky flag), and osk_comm_status says why.
    std::lock_guard<std::mutex> lc(comm->mu);
    std::lock_guard<std::mutex> lv(view->mu);
    rc = order_after_last(view, st);
    if (rc) return rc;
    // world > 1: the communicator's fixed block (the RCCL count is the same on every rank whatever the call
    // passes; a call that differs is caught by the header check).  A call beyond the limits sends a refusal
    // header (magic kXRefused) with empty lists, so every rank's reduce reports count −1 and no rank waits
    // alone in the all-gather; this rank returns OSK_ERR_INVALID after issuing it.
    const bool fixed = comm->world > 1;
    const bool refuse_local = !local_err.empty();   // (world > 1 here)
    const bool over = fixed && (refuse_local || n_queries > comm->dev_max_nq || k > comm->dev_max_k ||
                                shards_per_rank > comm->dev_max_spr);
    const Block B = fixed ? fixed_block_of(comm) : block_of(n_queries, k, shards_per_rank);
    uint64_t hw[kXHdrWords];
    header_words(hw, ++comm->seq, n_queries, k, from, size, shards_per_rank, view->dim, view->enc, comm->world);
    if (over) {
        hw[0] = kXRefused;
        OSK_HIP(view->ws_xkeys.reserve(sizeof(uint64_t) * B.words));
        OSK_HIP(hipMemsetAsync(view->ws_xkeys.p, 0, sizeof(uint64_t) * B.keys, st));
        OSK_HIP(launch_xhdr_fill(view->ws_xkeys.as<uint64_t>() + B.keys, hw, d_queries, 0, view->d_shard_index.as<int32_t>(),
                                 view->n_shards, std::min(view->n_shards, comm->dev_max_spr), st));
    } else if (comm->world == 1 && view->n_shards == shards_per_rank) {
        // world 1 with no padding: the lists are the whole image and there is no other rank's header to
        // compare, so neither the header nor the shard-index trailer is written (the reduce takes the view's
        // shard indices directly) — one launch less per call
        rc = search_padded(view, d_queries, n_queries, k, d_accept, shards_per_rank, st);
        if (rc) return rc;
    } else {
        rc = fill_block(view, d_queries, n_queries, k, d_accept, shards_per_rank, hw, st, fixed ? &B : nullptr);
        if (rc) return rc;
    }
    osk_view* const vs[1] = {view};
    const uint64_t* image = view->ws_xkeys.as<uint64_t>();
    if (comm->world > 1) {   // world 1: the local block is the whole image
        // block ready on st → the all-gather on the communicator's exchange stream → the reduce on st.
        // The view's next search (same view, any stream) is ordered after this call's reduce on st
        // (order_after_last), which waits for this gather, so ws_xkeys / ws_xgath are never raced.
        OSK_HIP(enter_xstream(comm, 0, st));
        rc = gather_blocks(comm, vs, B.words, comm->xstreams.data());
        if (rc) return rc;
        OSK_HIP(leave_xstream(comm, 0, st));
        image = view->ws_xgath.as<uint64_t>();
    }
    if (refuse_local) {
        set_error("osk_shards_search_merge_device: " + local_err +
                  " (refused on every rank: their reduce reports count -1, communicator poisoned)");
        return OSK_ERR_INVALID;
    }
    const int32_t* sidx = nullptr;
    XLayout x = image_layout(comm, image, B, &sidx);
    if (comm->world == 1 && !over && view->n_shards == shards_per_rank) {   // (no header written: see above)
        x.hdr = nullptr;
        x.si_stride = shards_per_rank;
        sidx = view->d_shard_index.as<int32_t>();
    }
    // (a refusing rank reduces with the limits' shape: its outputs are count −1 like every other rank's)
    OSK_HIP(launch_coord_reduce(image, nullptr, sidx, over ? std::min(n_queries, comm->dev_max_nq) : n_queries,
                               comm->world, over ? comm->dev_max_spr : shards_per_rank, over ? std::min(k, comm->dev_max_k) : k,
                               from, size, d_scores, d_docs, d_shard_out, d_count, d_total_hits, d_max_score, st, x));
    if (over) {
        set_error("osk_shards_search_merge_device: the call (n_queries " + std::to_string(n_queries) + ", k " +
                  std::to_string(k) + ", shards_per_rank " + std::to_string(shards_per_rank) +
                  ") exceeds the communicator's device limits (" + std::to_string(comm->dev_max_nq) + ", " +
                  std::to_string(comm->dev_max_k) + ", " + std::to_string(comm->dev_max_spr) +
                  "): refused on every rank (count -1), communicator poisoned; see osk_comm_set_device_limits");
        return OSK_ERR_INVALID;
    }
    return OSK_OK;
    OSK_GUARD_END
}

int32_t osk_comm_set_device_limits(osk_comm* comm, int32_t max_queries, int32_t max_k, int32_t max_shards_per_rank) {
    OSK_GUARD_BEGIN
    clear_error();
    OSK_REQUIRE(comm != nullptr, "null communicator");
    OSK_REQUIRE(max_queries >= 1 && max_k >= 1 && max_k <= OSK_MAX_K && max_shards_per_rank >= 1,
                "limits must be >= 1 (k <= OSK_MAX_K)");
    OSK_REQUIRE((int64_t)max_queries * max_k * max_shards_per_rank <= ((int64_t)1 << 27),
                "device limits: the exchange block would exceed 1 GiB");
    std::lock_guard<std::mutex> lc(comm->mu);
    comm->dev_max_nq = max_queries;
    comm->dev_max_k = max_k;
    comm->dev_max_spr = max_shards_per_rank;
    return OSK_OK;
    OSK_GUARD_END
}

int32_t osk_shards_search_merge(osk_comm* comm, osk_view* const* views, int32_t n_views, const void* queries,
                                int32_t n_queries, int32_t k, const uint64_t* const* accept, int32_t from, int32_t size,
                                float* out_scores, int32_t* out_docs, int32_t* out_shard_index, int32_t* out_count,
                                int64_t* out_total_hits, float* out_max_score) {
    OSK_GUARD_BEGIN
    clear_error();
    OSK_REQUIRE(comm != nullptr && views != nullptr && queries != nullptr, "null argument");
    OSK_REQUIRE(out_scores && out_docs && out_shard_index && out_count && out_total_hits && out_max_score,
                "null output");
    OSK_REQUIRE(n_views == (int32_t)comm->devices.size(), "need one view per local device of the communicator");
    int spr = 1;
    for (int i = 0; i < n_views; ++i) {
        OSK_REQUIRE(views[i] != nullptr, "null view");
        OSK_REQUIRE(views[i]->device == comm->devices[i], "view i must live on the communicator's local device i");
        OSK_REQUIRE(views[i]->dim == views[0]->dim && views[i]->enc == views[0]->enc,
                    "all views must share dim and encoding");
        spr = std::max(spr, views[i]->n_shards);
    }
    int32_t rc = check_merge_args(comm, n_queries, k, from, size, spr);
    if (rc) return rc;
    // (no refusal on the poison flag before the collectives: see osk_shards_search_merge_device)
    std::lock_guard<std::mutex> lc(comm->mu);
    std::vector<std::unique_lock<std::mutex>> locks;
    std::vector<hipStream_t> sts(n_views);
    const int64_t elem = views[0]->enc == ENC_FLOAT32 ? 4 : 1;
    const size_t qbytes = (size_t)n_queries * views[0]->dim * elem;
    size_t seg_off = 0;
    for (int i = 0; i < n_views; ++i) {
        osk_view* v = views[i];
        rc = check_device(v->device);
        if (rc) return rc;
        sts[i] = device_stream(v->device);
        locks.emplace_back(v->mu);
        rc = order_after_last(v, sts[i]);
        if (rc) return rc;
        // queries and accept bitsets → this device
        OSK_HIP(v->ws_qin.reserve(std::max<size_t>(16, qbytes)));
        OSK_HIP(hipMemcpyAsync(v->ws_qin.p, queries, qbytes, hipMemcpyHostToDevice, sts[i]));
        const int ns = (int)v->segs.size();
        const uint64_t* const* d_acc = nullptr;
        bool any = false;
        for (int j = 0; accept && j < ns; ++j) any |= accept[seg_off + j] != nullptr;
        if (any) {
            size_t words = 0;
            for (int j = 0; j < ns; ++j)
                if (accept[seg_off + j]) words += (size_t)(v->segs[j]->max_doc + 63) / 64;
            OSK_HIP(v->ws_accept.reserve(std::max<size_t>(8, words * 8)));
            OSK_HIP(v->ws_accept_ptrs.reserve(sizeof(void*) * ns));
            std::vector<const uint64_t*> ptrs(ns, nullptr);
            size_t off = 0;
            for (int j = 0; j < ns; ++j) {
                if (!accept[seg_off + j]) continue;
                const size_t w = (size_t)(v->segs[j]->max_doc + 63) / 64;
                ptrs[j] = v->ws_accept.as<uint64_t>() + off;
                OSK_HIP(hipMemcpyAsync(const_cast<uint64_t*>(ptrs[j]), accept[seg_off + j], w * 8,
                                       hipMemcpyHostToDevice, sts[i]));
                off += w;
            }
            OSK_HIP(hipMemcpyAsync(v->ws_accept_ptrs.p, ptrs.data(), sizeof(void*) * ns, hipMemcpyHostToDevice,
                                   sts[i]));
            OSK_HIP(hipStreamSynchronize(sts[i]));   // ptrs is a local
            d_acc = v->ws_accept_ptrs.as<const uint64_t*>();
        }
        seg_off += ns;
        OSK_HIP(v->ws_keys.reserve(sizeof(uint64_t) * (size_t)n_queries * v->n_shards * k));
        OSK_HIP(v->ws_counts.reserve(sizeof(int32_t) * (size_t)n_queries * v->n_shards));
        rc = view_search_device(v, v->ws_qin.p, n_queries, k, d_acc, v->ws_keys.as<uint64_t>(),
                                v->ws_counts.as<int32_t>(), nullptr, sts[i]);
        if (rc) return rc;
    }
    // the call agreement (fixed-size headers, shards per rank) while the scans run: a rank that issued
    // another call is caught before the variable-size block gather (agree_call)
    if (comm->world > 1) {
        rc = agree_call(comm, views, n_queries, k, from, size, &spr);
        if (rc) {
            for (int i = 0; i < n_views; ++i) {   // the scans already issued write the views' workspaces
                (void)hipSetDevice(views[i]->device);
                (void)hipStreamSynchronize(sts[i]);
            }
            return rc;
        }
    }
    const Block B = block_of(n_queries, k, spr);
    uint64_t hw[kXHdrWords];
    header_words(hw, ++comm->seq, n_queries, k, from, size, spr, views[0]->dim, views[0]->enc, comm->world);
    for (int i = 0; i < n_views; ++i) {
        osk_view* v = views[i];
        OSK_HIP(hipSetDevice(v->device));
        OSK_HIP(v->ws_xkeys.reserve(sizeof(uint64_t) * B.words));
        OSK_HIP(launch_xhdr_fill(v->ws_xkeys.as<uint64_t>() + B.keys, hw, v->ws_qin.p, (int64_t)qbytes,
                                 v->d_shard_index.as<int32_t>(), v->n_shards, spr, sts[i]));
        rc = pad_lists(v, n_queries, k, spr, sts[i]);
        if (rc) return rc;
    }
    const uint64_t* image = views[0]->ws_xkeys.as<uint64_t>();
    if (comm->world > 1) {
        for (int i = 0; i < n_views; ++i) {
            OSK_HIP(hipSetDevice(views[i]->device));
            OSK_HIP(enter_xstream(comm, i, sts[i]));
        }
        rc = gather_blocks(comm, views, B.words, comm->xstreams.data());
        if (rc) return rc;
        for (int i = 0; i < n_views; ++i) {   // every view's next search reuses its ws_xkeys / ws_xgath
            OSK_HIP(hipSetDevice(views[i]->device));
            OSK_HIP(leave_xstream(comm, i, sts[i]));
        }
        image = views[0]->ws_xgath.as<uint64_t>();
    }
    // the coordinator reduce on local device 0 (every local device holds the same image)
    osk_view* v0 = views[0];
    OSK_HIP(hipSetDevice(v0->device));
    const size_t n_out = (size_t)n_queries * size;
    const size_t b_sc = n_out * 4, b_doc = n_out * 4, b_sh = n_out * 4, b_cnt = (size_t)n_queries * 4,
                 b_tot = (size_t)n_queries * 8, b_max = (size_t)n_queries * 4;
    const size_t o_sc = 0, o_doc = o_sc + b_sc, o_sh = o_doc + b_doc, o_cnt = o_sh + b_sh,
                 o_tot = (o_cnt + b_cnt + 7) / 8 * 8, o_max = o_tot + b_tot, total_b = o_max + b_max;
    OSK_HIP(v0->ws_xout.reserve(total_b));
    char* ob = v0->ws_xout.as<char>();
    const int32_t* sidx = nullptr;
    const XLayout x = image_layout(comm, image, B, &sidx);
    OSK_HIP(launch_coord_reduce(image, nullptr, sidx, n_queries, comm->world, spr, k, from, size,
                               reinterpret_cast<float*>(ob + o_sc), reinterpret_cast<int32_t*>(ob + o_doc),
                               reinterpret_cast<int32_t*>(ob + o_sh), reinterpret_cast<int32_t*>(ob + o_cnt),
                               reinterpret_cast<int64_t*>(ob + o_tot), reinterpret_cast<float*>(ob + o_max), sts[0], x));
    OSK_HIP(v0->h_stage.reserve(total_b));
    OSK_HIP(hipMemcpyAsync(v0->h_stage.p, ob, total_b, hipMemcpyDeviceToHost, sts[0]));
    for (int i = 0; i < n_views; ++i) {
        OSK_HIP(hipSetDevice(views[i]->device));
        OSK_HIP(hipStreamSynchronize(sts[i]));
    }
    rc = poisoned(comm);   // the ranks issued different calls: no result
    if (rc) return rc;
    const char* hb = static_cast<const char*>(v0->h_stage.p);
    std::memcpy(out_scores, hb + o_sc, b_sc);
    std::memcpy(out_docs, hb + o_doc, b_doc);
    std::memcpy(out_shard_index, hb + o_sh, b_sh);
    std::memcpy(out_count, hb + o_cnt, b_cnt);
    std::memcpy(out_total_hits, hb + o_tot, b_tot);
    std::memcpy(out_max_score, hb + o_max, b_max);
    return OSK_OK;
    OSK_GUARD_END
}

}  // extern "C"
