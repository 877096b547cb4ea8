/*
 * osknn.h — C-ABI of libosknn.so, the MI355X-native exact k-NN scoring path for OpenSearch.
 *
 * This is the drop-in boundary. Every entry point is `extern "C"`, takes plain pointers and
 * sizes, never throws, never aborts, and is safe to call from many threads at once (OpenSearch's
 * `search` and `index_searcher` pools, S/threadpool/ThreadPool.java:106,126). Errors are returned
 * as negative codes; the message of the last error on the calling thread is `osk_last_error()`.
 * A Java caller maps a negative code to an IOException, which OpenSearch turns into a shard
 * failure (S/search/query/QueryPhase.java:307-309) — the library never brings the node down.
 *
 * Concurrency:
 *   - host entries (osk_seg_search, osk_view_search): every concurrent call leases a workspace slot of
 *     the view (the view itself, or a replica view over the same segments, created on demand, at most
 *     8) together with that slot's own stream, so concurrent synchronous searches of one segment or
 *     shard set run concurrently on the device; a call waits only when all 8 slots are busy.
 *     osk_shards_search_merge instead takes each view's own workspace under its mutex, on the library's
 *     stream (one collective sequence per communicator serialises those calls anyway).  Concurrent unfiltered calls with the same k /
 *     from / size are moreover batched opportunistically: while a batch runs, the calls that arrive
 *     queue up and the next batch takes them all (≤ 32 queries, one corpus pass for all of them;
 *     results identical to unbatched calls; tune "host_batching", "host_batch_leaders");
 *   - device entries (osk_view_search_device, osk_shards_search_merge_device) run on the caller's
 *     stream with the view's own workspace: calls on one view are serialised by its mutex, and a
 *     search whose stream differs from the previous search's first waits for the work already
 *     enqueued on that stream, so a caller stream must stay valid until the next search on the view
 *     has been issued, or the view released.  Callers that want device-side concurrency create one
 *     view per search thread over the same segments (views share the segments' HBM).
 *
 * Citation convention: `S/` = /root/reference/server/src/main/java/org/opensearch/ ;
 * [L] = behaviour of the un-vendored lucene-core 10.3.0 jar (gradle/libs.versions.toml:3) whose
 * interface is evidenced by the reference call site given next to it.
 *
 * What each entry point replaces in the reference stack:
 *
 *   osk_seg_stage / osk_seg_stage_device / osk_seg_synth
 *       [L] KnnVectorsFormat.fieldsReader(SegmentReadState) → the reader's constructor / warm step:
 *       one segment's flat vector values (.vec, row-major little-endian) staged ONCE into HBM.
 *       Segment open: S/index/engine/InternalEngine.java:584-589; warmers
 *       S/index/engine/InternalEngine.java:2409-2432; codec choice S/index/codec/CodecService.java:70-99.
 *   osk_seg_release
 *       [L] KnnVectorsReader.close() — when the segment is merged away / its refcount drops to 0.
 *   osk_seg_search
 *       [L] KnnVectorsReader.search(String field, float[]|byte[] target, KnnCollector, AcceptDocs)
 *       reached through LeafReader.searchNearestVectors (4-arg 10.3 signature evidenced at
 *       S/index/engine/TranslogLeafReader.java:379-386). Exact (brute-force) top-k over the
 *       segment with Lucene's exact-search semantics: score desc, ties → lower doc.
 *   osk_view_create / osk_view_search / osk_view_search_device
 *       A shard's leaves (and several shards on one GPU): the per-leaf exact search that
 *       [L] AbstractKnnVectorQuery.rewrite runs for every leaf from
 *       S/search/internal/ContextIndexSearcher.java:203-218, the per-leaf TopDocs.merge(k, …)
 *       into the shard's top-k, and the shard collector's cut to from+size
 *       (S/search/query/TopDocsCollectorContext.java:866-891).
 *   osk_merge_device / osk_topdocs_merge
 *       The coordinator's reduce: S/action/search/SearchPhaseController.java:224-246 (mergeTopDocs →
 *       [L] TopDocs.merge(from, size, shardHits): score desc, then shardIndex asc, then doc asc),
 *       :248-253 (setShardIndex) and TopDocsStats (:839-901: Σ totalHits, max maxScore).
 *       osk_merge_device runs on the GPU after the RCCL all-gather of per-shard top-k lists;
 *       osk_topdocs_merge is the same reduce over host arrays (no device needed).
 */
#ifndef OSKNN_H
#define OSKNN_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OSK_ABI_VERSION 2
#define OSK_MAX_K       10000 /* largest k: index.max_result_window (S/index/IndexSettings.java:223-226) */
#define OSK_MAX_DIM     4096

/* ---- return codes ---- */
#define OSK_OK               0
#define OSK_ERR_INVALID     -1   /* bad argument (null pointer, k <= 0, dim mismatch, ...) */
#define OSK_ERR_DEVICE      -2   /* a HIP runtime call failed */
#define OSK_ERR_OOM         -3   /* device or host allocation failed */
#define OSK_ERR_UNSUPPORTED -4   /* valid request this build does not implement */
#define OSK_ERR_NO_DEVICE   -5   /* no usable gfx950 device */

/* ---- [L] VectorEncoding ---- */
#define OSK_FLOAT32 0
#define OSK_BYTE    1

/* ---- [L] VectorSimilarityFunction (ordinal order of the Lucene enum) ---- */
#define OSK_EUCLIDEAN             0
#define OSK_DOT_PRODUCT           1
#define OSK_COSINE                2
#define OSK_MAXIMUM_INNER_PRODUCT 3

/* ---- synthetic corpus distributions (bench / tests) ---- */
#define OSK_DIST_UNIFORM01      0   /* U[0,1)                         (C1)            */
#define OSK_DIST_UNIFORM01_X128 1   /* U[0,1)·128, SIFT-like          (C2)            */
#define OSK_DIST_NORMALISH      2   /* Irwin–Hall(4) ≈ N(0,1)                          */
#define OSK_DIST_NORMALISH_UNIT 3   /* Irwin–Hall(4), each row L2-normalised (C3, C4)  */
#define OSK_DIST_INT8           4   /* U{-128..127} bytes             (C5 int8)        */

typedef struct osk_seg  osk_seg;   /* one segment's vector field, resident in HBM */
typedef struct osk_view osk_view;  /* the segments of one or more shards on ONE device */

int32_t     osk_abi_version(void);
/* Message of the last failed call on this thread ("" if none). Valid until the next call. */
const char* osk_last_error(void);
int32_t     osk_device_count(int32_t* n);

/* Stage one segment into HBM on `device`.
 *   rows        host, n_rows × dim elements row-major (f32 or int8 per `encoding`), ord order
 *   ord_to_doc  NULL = dense (doc == ord), else n_rows ascending segment-local docIDs
 *   max_doc     the leaf's maxDoc (bounds the accept bitset); must be ≥ the largest doc + 1
 * The rows are copied; the caller's buffer may be freed on return. */
int32_t osk_seg_stage(int32_t device, const void* rows, int64_t n_rows, int32_t dim,
                      int32_t encoding, int32_t similarity, const int32_t* ord_to_doc,
                      int32_t max_doc, osk_seg** out);
/* Same, from rows already on `device` (row pitch `src_pitch_bytes`); ord_to_doc is host memory.
 * The copy is issued on the library's own stream for `device`, which does not wait on the caller's
 * streams: whatever writes d_rows must have completed (e.g. its stream synchronised) before the call. */
int32_t osk_seg_stage_device(int32_t device, const void* d_rows, int64_t src_pitch_bytes,
                             int64_t n_rows, int32_t dim, int32_t encoding, int32_t similarity,
                             const int32_t* ord_to_doc, int32_t max_doc, osk_seg** out);
/* Same, from a Lucene99 flat vectors data file (.vec): the field's rows are the n_rows × dim
 * little-endian elements at byte data_offset (its FieldEntry in .vemf: vectorDataOffset), memory-mapped
 * and staged through pinned buffers into HBM (S/index/store/FsDirectoryFactory.java:98-110 maps .vec;
 * S/index/IndexModule.java:215-233).  ord_to_doc as osk_seg_stage (the docsWithField IndexedDISI's
 * order for a sparse field).  A missing or short file is OSK_ERR_INVALID with the OS message. */
int32_t osk_seg_stage_file(int32_t device, const char* path, int64_t data_offset, int64_t n_rows, int32_t dim,
                           int32_t encoding, int32_t similarity, const int32_t* ord_to_doc, int32_t max_doc,
                           osk_seg** out);
/* A synthetic dense segment generated on the device: row r of the segment is global row
 * row0 + r of the counter-based generator (seed, dist). osk_synth_host() yields identical values. */
int32_t osk_seg_synth(int32_t device, int64_t n_rows, int32_t dim, int32_t encoding,
                      int32_t similarity, uint64_t seed, int32_t dist, int64_t row0,
                      osk_seg** out);
/* Segments are reference counted: the stage/synth call returns one reference, every view created over
 * the segment holds another (so a segment merged away or closed under a live view stays valid until
 * the view is released).  osk_seg_retain adds a reference; osk_seg_release drops one and frees the
 * HBM copy at zero. */
int32_t osk_seg_release(osk_seg* seg);
int32_t osk_seg_retain(osk_seg* seg);
/* HBM bytes the segment owns now: rows, norms, doc map and every derived copy built so far. */
int32_t osk_seg_footprint(const osk_seg* seg, int64_t* hbm_bytes);
/* Build derived copies ahead of the first search that needs them (the warmer's job,
 * S/index/engine/InternalEngine.java:2409-2432, S/index/IndexWarmer.java:132-135).  Float32 segments
 * get the prefilter copy at staging; the other two are built here or, if never warmed, by the first
 * search that takes their path.  No-op for byte fields. */
#define OSK_WARM_PREFILTER      1   /* int8 copy + 16-B bound terms per row (¼ + 16 B of the rows), and
                                       for dims ≥ 512 the 6-bit tier of single queries (+ ≈3/16 + 16 B)   */
#define OSK_WARM_PREFILTER_MFMA 2   /* its 16-row tiled twin read by the batched int8 MFMA prefilter    */
#define OSK_WARM_BATCHED        4   /* bf16 hi/lo split copy of the batched bf16×3 MFMA path (= rows)   */
#define OSK_WARM_ALL            7
int32_t osk_seg_warm(osk_seg* seg, int32_t what);
int32_t osk_seg_info(const osk_seg* seg, int64_t* n_rows, int32_t* dim, int32_t* encoding,
                     int32_t* similarity, int32_t* max_doc, int32_t* device);

/* Host generator behind osk_seg_synth (f32 out for dists 0-3, int8 out for dist 4). */
int32_t osk_synth_host(void* out, int64_t row0, int64_t n_rows, int32_t dim, uint64_t seed,
                       int32_t dist);

/* [L] KnnVectorsReader.search — exact top-k of one segment, host buffers, synchronous.
 *   queries      n_queries × dim (f32 or int8, the segment's encoding)
 *   accept_bits  NULL = all docs; else ceil(max_doc/64) words, LSB-first, bit d = doc d accepted
 *                (Lucene AcceptDocs = liveDocs ∩ filter)
 *   out_scores/out_docs  n_queries × k, per query score desc then doc asc; slots past
 *                out_count[q] are score = -inf, doc = INT32_MAX
 *   out_visited  (optional) number of vectors scored = KnnCollector.visitedCount()
 * 1 ≤ k ≤ OSK_MAX_K. */
int32_t osk_seg_search(osk_seg* seg, const void* queries, int32_t n_queries, int32_t k,
                       const uint64_t* accept_bits, float* out_scores, int32_t* out_docs,
                       int32_t* out_count, int64_t* out_visited);

/* Group segments into shards on one device.
 *   seg_shard[i]     which shard (0 … n_shards-1) segment i belongs to
 *   seg_doc_base[i]  the leaf's docBase inside its shard (LeafReaderContext.docBase)
 *   shard_index[s]   the coordinator's shardIndex of shard s (rank in sorted ShardId order,
 *                    S/action/search/TransportSearchAction.java:1188,
 *                    S/cluster/routing/GroupShardsIterator.java:59-62); NULL = 0 … n_shards-1
 * All segments must share device, dim, encoding and similarity. */
int32_t osk_view_create(osk_seg* const* segs, int32_t n_segs, const int32_t* seg_shard,
                        const int32_t* seg_doc_base, int32_t n_shards,
                        const int32_t* shard_index, osk_view** out);
int32_t osk_view_release(osk_view* view);
/* osk_seg_warm of every segment plus the view's own tables for those paths. */
int32_t osk_view_warm(osk_view* view, int32_t what);

/* Per-shard exact top-k on the device, asynchronous on `stream` (NULL = the library's stream for
 * the device). All buffers are DEVICE pointers:
 *   d_queries      n_queries × dim
 *   d_accept       NULL, or a device array of n_segs device pointers (each NULL or a bitset)
 *   d_shard_keys   out, n_queries × n_shards × k uint64 "hit keys", best first, 0 = empty slot:
 *                  key = (sortable(score) << 32) | (0xFFFFFFFF - doc), doc = shard-local docID
 *   d_shard_counts out, n_queries × n_shards hits per shard (≤ k)
 *   d_visited      optional out, n_segs int64 (vectors scored per segment, per query) */
int32_t osk_view_search_device(osk_view* view, const void* d_queries, int32_t n_queries,
                               int32_t k, const uint64_t* const* d_accept, uint64_t* d_shard_keys,
                               int32_t* d_shard_counts, int64_t* d_visited, void* stream);

/* Coordinator reduce on the device over per-shard lists laid out as osk_view_search_device
 * writes them (possibly all-gathered from several GPUs: n_shards = all shards).
 *   d_shard_index  n_shards shardIndex values (device)
 *   top-docs size per shard = min(k, from+size) (the shard collector's cut)
 *   outputs (device): n_queries × size scores/docs/shard indices, per-query count,
 *   total hits (Σ shard hits) and max score (NaN if no hits). */
int32_t osk_merge_device(int32_t device, const uint64_t* d_shard_keys,
                         const int32_t* d_shard_counts, const int32_t* d_shard_index,
                         int32_t n_queries, int32_t n_shards, int32_t k, int32_t from,
                         int32_t size, float* d_scores, int32_t* d_docs, int32_t* d_shard_out,
                         int32_t* d_count, int64_t* d_total_hits, float* d_max_score,
                         void* stream);

/* The same reduce straight over an all-gather's output (no counts, no re-layout): per-rank lists
 * [n_queries][shards_per_rank][k] concatenated rank after rank, i.e. shard s = r·shards_per_rank + j
 * of query q at ((r·n_queries + q)·shards_per_rank + j)·k.  A list's hits are its non-zero keys
 * (best first, zero-padded, as osk_view_search_device writes them).  d_shard_index has
 * n_ranks·shards_per_rank entries. */
int32_t osk_merge_device_ranked(int32_t device, const uint64_t* d_keys, int32_t n_ranks,
                                int32_t shards_per_rank, const int32_t* d_shard_index, int32_t n_queries,
                                int32_t k, int32_t from, int32_t size, float* d_scores, int32_t* d_docs,
                                int32_t* d_shard_out, int32_t* d_count, int64_t* d_total_hits,
                                float* d_max_score, void* stream);

/* Scan-kernel timing (benchmarks): osk_view_profile(view, N) resets and, for N > 0, samples every N-th
 * osk_view_search_device call (N = 1: every call; 0: off); osk_view_scan_time then reads the summed
 * duration of the sampled calls' scan launches (HIP start/stop events stamped by the launches on the
 * call's stream) and the number of sampled calls.  A sampled call pays a few µs of stream time for the
 * stamps; keep it off in production. */
int32_t osk_view_profile(osk_view* view, int32_t enable);
int32_t osk_view_scan_time(osk_view* view, double* total_ms, int64_t* calls);

/* Process-wide tuning knobs (atomic; a search reads each knob once, and every setting returns the same
 * exact results — only speed changes):
 *   "scan_nt"         0|1 non-temporal corpus loads in the streaming scan (default 1)
 *   "tiles_target"    workgroup tiles per view for the scans (default 0 = whole rounds of the chip's
 *                     resident slots; at view create)
 *   "tile_slots_per_cu", "tile_max_rounds"  ...its resident workgroups per CU (4) and rounds cap (4)
 *   "tile_min_rows"   ...with at least this many rows per tile (default 1024; at view create)
 *   "tile_large_slots" views of >= CUs x this x tile_min_rows rows get CUs x this tiles (24; 0 = off)
 *   "tile_large_slots_512" the same for views of >= 512-dim rows (12)
 *   "mfma_min_batch"  batches of at least this many float32 queries (and k ≤ 12) may take the bf16×3
 *                     MFMA path (default 96; 0 = never)...
 *   "sq8_cost_pct"    ...when its 256-query blocks cost no more than the int8 prefilter's launches for
 *                     the same queries, by a per-row cost model of both measured on MI355X with the
 *                     prefilter's side scaled by this / 100 (default 100)
 *   "mfma_units"      workgroup units of the MFMA candidate pass per view (default 0: 256 below
 *                     16384 tiles of 128 rows, else 512)
 *   "sq8"             0|1 certified int8 prefilter for float32 searches with k ≤ 12 that do not take
 *                     the bf16×3 path (default 1; results are bit-identical either way)
 *   "sq6"             0|1 single unfiltered prefiltered queries scan the 6-bit tier where the view has
 *                     one (dims ≥ 512; default 1) instead of the int8 copy...
 *   "sq6_probe_pct"   ...unless the view's first 4 such calls re-bound more than this % of the rows from
 *                     the int8 copy (default 10; the view then keeps the int8 tier)
 *   "sq8_mfma_min"    prefilter batches of at least this many queries scan on int8 MFMA (sq8_mfma,
 *                     default 2; 0 = always the VALU sq8_scan)
 *   "sq8_mfma_queries"  16 | 32 queries per sq8_mfma launch (default 32)
 *   "host_batching"   0|1 opportunistic batching of concurrent unfiltered host calls (default 1)
 *   "host_batch_leaders"  batches of host calls in flight per view (default 1; more overlap, smaller
 *                     batches)
 *   "sq8_mfma_nt"     0|1 non-temporal row loads in sq8_mfma (default 1)
 *   "sq8_mfma_ring"   LDS-DMA ring slots per wave in sq8_mfma for rows of ≤ 256 dims (default -1 = as many
 *                     as keep 4 workgroups per CU, 0 = register row loads)
 *   "i8_stream"       0|1 single unfiltered byte-vector queries on scan_i8_stream (default 1) or scan_i8
 *   "filter_gather"   0|1 filtered prefilter scans over the device-compacted accepted ordinals
 *                     (osk_filter.hip; default 1) instead of a walk over 64-row bitset windows
 *   "gather_min"      accepted rows per gather tile at least (default 0 = every tile of the segment)
 *   "select_mid_k"    0|1 float32 searches with 12 < k ≤ 64 take the select path over int8 bounds
 *                     (default 1) instead of the fp32 streaming scan; k > 64 always takes it
 *   "call_timing"     0|1 host entries time each call on the device (osk_last_call_device_ns; default 0)
 *   "sel_writer"      select path bounds writer: 0 = 4 row groups in flight + Java's transform,
 *                     1 = 4 groups + fp32 COSINE bounds, 2 = 2 groups (default), 3 = 1 group (fast bounds)
 *   "sq8_wide_min"    unfiltered prefilter batches of at least this many queries may take the wide int8
 *                     kernels (256 queries per corpus pass; default 64; 0 = never)
 *   "sq8_wide_rows"   0|1 rows of ≤ 128 dims: the wide pilot and main passes on sq8_wide_rows, without a step
 *                     barrier (default 1) instead of the ring kernel sq8_wide
 *   "sq8_wide_rows_claim"  0|1 its waves claim 16-row groups from a per-quarter counter (default 1) or take
 *                     the fixed interleave
 *   "sq8_wide_phase"  the wide main pass's first launch covers 1/this of the quarters (default 8)
 *   "sq8_wide_pilot_rows"  wide pilot rows per quarter (default 0 = 128, 256 at ≥ 512 dims, raised to
 *                     sample ≥ 64k rows per shard)
 *   "sq8_wide_quarter_rows"  rows per wide quarter (default 0 = auto, ≤ 16,384; at the view's first wide batch)
 *   "sq8_scan_deep"   0|1 single-query sq8_scan over ≤ 256 dims with 8 row groups in flight per wave
 *                     (default 0: measured slower)
 * The testing build (libosknn_testing.so) also accepts "sq8_mfma_ablate", "mfma_ablate" (A/B timing,
 * results wrong), "sq8_force_fallback" (every prefilter list re-scanned exactly) and "settle_trace";
 * the shipped library returns OSK_ERR_UNSUPPORTED for them. */
int32_t osk_tune_set(const char* key, int64_t value);

/* Batched-path counters of a view: searches that took the MFMA path, and queries among them whose
 * certificate failed and were recomputed by the exact streaming scan. */
int32_t osk_view_stats(osk_view* view, int64_t* batched_calls, int64_t* fallback_queries);
/* Named counters of a view: "mfma_calls", "mfma_fallback_queries" (as osk_view_stats),
 * "sq8_calls" (prefiltered searches), "sq6_calls" (those whose scan read the 6-bit tier),
 * "sq6_rebound_rows" (rows the 6-bit scan re-bounded from the int8 copy, all calls),
 * "sq8_fallback_queries" (queries where some tile's candidate
 * list overflowed past the certificate and the tile was re-scanned exactly), "sq8_exact_tiles"
 * (such tiles), "sq8_rescored_rows" (rows re-scored exactly, all calls), "select_calls" (searches
 * on the select path, k > 12), "host_slots" (workspace slots the host entries have leased: 1 + replicas),
 * "host_batches" / "host_batched_requests" (opportunistic batching of concurrent host calls).  The
 * search counters sum over the view and the replica slots its host entries leased.  osk_view_profile /
 * osk_view_scan_time time the device-entry calls on this view object only (per-call host timing:
 * osk_last_call_device_ns). */
int32_t osk_view_counter(osk_view* view, const char* name, int64_t* value);
/* Testing build only (the shipped library returns OSK_ERR_UNSUPPORTED): copy `bytes` of an internal
 * buffer of the view's last search ("akeys", "cand_a", "flags", "qsplit", "qnorm", "sq8cand", "sq8lb",
 * "qc", "settle_trace") to host memory. */
int32_t osk_view_debug_copy(osk_view* view, const char* name, void* host, int64_t bytes);

/* Device time of this thread's last synchronous host search (osk_seg_search / osk_view_search), for a
 * plugin's query-profile metrics: k-NN work shows up in the shard profile's rewrite time
 * (S/search/internal/ContextIndexSearcher.java:207-216) and a plugin adds its own timers through
 * SearchPlugin.getQueryProfileMetricsProvider (S/plugins/SearchPlugin.java:108).  Needs the
 * "call_timing" knob (osk_tune_set, off by default: two events per call).  *device_ns = nanoseconds from
 * the call's first to its last device operation on its stream (−1: timing off, or no host search on this
 * thread yet); *shared_by (optional) = how many concurrent host requests that launch chain served
 * (opportunistic batching: the time is shared by them). */
int32_t osk_last_call_device_ns(int64_t* device_ns, int32_t* shared_by);

/* Host-buffer convenience: shard search + coordinator merge on one device, synchronous.
 * accept: NULL or n_segs host pointers (each NULL or a host bitset). */
int32_t osk_view_search(osk_view* view, const void* queries, int32_t n_queries, int32_t k,
                        int32_t from, int32_t size, const uint64_t* const* accept,
                        float* out_scores, int32_t* out_docs, int32_t* out_shard_index,
                        int32_t* out_count, int64_t* out_total_hits, float* out_max_score);

/* [L] TopDocs.merge(from, size, shardHits) + TopDocsStats over host arrays (no device).
 *   shard_counts[s] hits of list s; shard_scores/shard_docs row s holds them at offset s*stride
 *   (each already sorted score desc, doc asc, as a shard returns them).
 *   The shardIndex of a hit is hit_shard_index[s*stride+i] when that array is given (lists that
 *   are themselves partial merges, S/action/search/QueryPhaseResultConsumer.java:212-277), else
 *   shard_index[s], else s. */
int32_t osk_topdocs_merge(int32_t n_shards, const int32_t* shard_counts, const float* shard_scores,
                          const int32_t* shard_docs, int32_t stride, const int32_t* shard_index,
                          const int32_t* hit_shard_index, int32_t from, int32_t size, float* out_scores, int32_t* out_docs,
                          int32_t* out_shard_index, int32_t* out_count, int64_t* out_total_hits,
                          float* out_max_score);

/* Decode hit keys (host). */
int32_t osk_decode_keys(const uint64_t* keys, int64_t n, float* scores, int32_t* docs);

/* Shard-result wire format (host, no device): S/common/lucene/Lucene.java:407-447 writeTopDocs for a
 * plain TopDocs (type byte 0 — what the shard collector of a k-NN DocAndScoreQuery returns):
 *   byte 0 | vLong total_hits | vInt relation | int32 BE floatToIntBits(max_score) | vInt n |
 *   n × (vInt doc, int32 BE floatToIntBits(score))
 * with StreamOutput's encodings (libs/core/.../io/stream/StreamOutput.java:247-337,480-482).
 *   relation  [L] TotalHits.Relation ordinal: 0 = EQUAL_TO, 1 = GREATER_THAN_OR_EQUAL_TO
 *   out       NULL (cap 0) = size query only; *out_len = the encoded size either way
 * total_hits < 0 fails like StreamOutput.writeVLong ("Negative longs unsupported, …"). */
int32_t osk_topdocs_write(int64_t total_hits, int32_t relation, float max_score, int32_t n,
                          const int32_t* docs, const float* scores, uint8_t* out, int64_t cap,
                          int64_t* out_len);
/* Lucene.readTopDocs (:314-357) for type 0; types 1/2 (field-sorted / collapsed docs, never a k-NN
 * shard result) → OSK_ERR_UNSUPPORTED; malformed input (unknown type, invalid vInt/vLong, bad
 * relation ordinal, negative count, truncation) → OSK_ERR_INVALID with StreamInput's message.
 * *consumed (optional) = bytes read. */
int32_t osk_topdocs_read(const uint8_t* buf, int64_t len, int64_t* total_hits, int32_t* relation,
                         float* max_score, int32_t cap_hits, int32_t* n, int32_t* docs, float* scores,
                         int64_t* consumed);

/* ---- multi-GPU (one node): shards ↔ GPUs, ONE RCCL all-gather of per-shard top-k, device merge ----
 * Replaces the coordinator's shard fan-out and reduce for shards that live on this node's GPUs:
 * S/action/search/AbstractSearchAsyncAction.java:262-268 (one request per shard copy, loop index =
 * shardIndex), S/action/search/SearchPhaseController.java:224-253 (mergeTopDocs → [L] TopDocs.merge
 * over the shards' results, setShardIndex) and :839-901 (TopDocsStats).  RCCL (librccl.so.1) is
 * loaded at first use; without it these entry points return OSK_ERR_UNSUPPORTED. */
#define OSK_COMM_ID_BYTES 128
typedef struct osk_comm osk_comm;

/* A fresh communicator id: call on ONE rank and hand the bytes to every rank out of band. */
int32_t osk_comm_unique_id(uint8_t* id /* OSK_COMM_ID_BYTES */);
/* One process per GPU: this process's rank of `world` on `device` (ncclCommInitRank; blocks until
 * every rank has joined). */
int32_t osk_comm_init_rank(int32_t device, int32_t rank, int32_t world, const uint8_t* id, osk_comm** out);
/* One process driving several GPUs (a JVM owning the node's GPUs): local device i is rank i. */
int32_t osk_comm_init_all(const int32_t* devices, int32_t n, osk_comm** out);
int32_t osk_comm_release(osk_comm* comm);
int32_t osk_comm_info(const osk_comm* comm, int32_t* rank, int32_t* world, int32_t* n_local);
/* Raw all-gather of `bytes` per rank (device buffers; one-device-per-process communicators). */
int32_t osk_comm_all_gather(osk_comm* comm, const void* d_send, void* d_recv, int64_t bytes, void* stream);

/* Every rank must issue the same searches in the same order (one collective sequence per communicator,
 * like the coordinator's one request per shard copy).  Each call's exchange block carries a header — call
 * sequence number, batch, k, from/size, shards per rank, dim/encoding and a fingerprint of the query
 * bytes — and the shard indices of the rank's lists, which the device reduce compares across ranks.
 * Ranks whose calls differ get count = −1 (and total hits −1) for every query of that call, and the
 * communicator becomes poisoned (sticky): every later call still issues its collective — a refusal based
 * on a flag the previous call's reduce writes asynchronously could differ between ranks and leave one
 * rank inside the all-gather forever — but its reduce reports count −1, and the synchronous host entry
 * returns OSK_ERR_INVALID (release and re-create the communicator).  The batch, k and shards per rank size
 * the all-gather, and RCCL requires every rank to pass the same count: the host entry agrees on a
 * fixed-size call header first and refuses on every rank together when they differ; the device entry
 * never waits on the host, so at world > 1 its all-gather moves a block of the communicator's FIXED size
 * (osk_comm_set_device_limits) whatever the call's batch, k and shards per rank, and its header check
 * catches every difference — batch, k and shards per rank included.  osk_comm_status reports the flag (OSK_ERR_INVALID + message) without
 * synchronising: synchronise the call's stream first.  info (optional, 4 values): [flag, rank 0's call
 * number, first differing rank, its call number].  (A rank that never issues its call leaves the others
 * blocked inside RCCL, as the coordinator would wait on a shard that never answers.) */
int32_t osk_comm_status(const osk_comm* comm, int64_t* info);
/* The device entry's exchange limits (osk_shards_search_merge_device at world > 1): its all-gather moves
 * max_queries × max_shards_per_rank × max_k keys plus the header per rank and call, so the RCCL count is a
 * property of the communicator, equal on every rank by construction, and ranks whose calls differ in
 * batch, k or shards per rank get count −1 from the header check instead of an all-gather of mismatched
 * counts (undefined under RCCL: a hang).  Set them once, identically on every rank (like world and id),
 * before the first device call, to the largest batch, k and shards per rank the node will issue (the
 * block size is the price of every call: 1 × 10 × 1 keys for single-query k = 10 search at one shard per
 * GPU).  Defaults: 1 query, k 100, 8 shards per rank.  A call beyond the limits still issues its
 * collective with a refusal header (the other ranks must not wait alone): every rank's reduce reports
 * count −1, the communicator is poisoned, and this rank's call returns OSK_ERR_INVALID.  World 1 runs no
 * collective; the limits do not apply there. */
int32_t osk_comm_set_device_limits(osk_comm* comm, int32_t max_queries, int32_t max_k, int32_t max_shards_per_rank);
/* Testing build only (libosknn_testing.so; the shipped library returns OSK_ERR_UNSUPPORTED): a
 * communicator of `world` processes that may share ONE device (RCCL refuses that), whose all-gather
 * goes through the POSIX shared-memory segment named by id (a NUL-terminated "/name"), at most
 * slot_bytes per rank and call.  It drives exactly the world > 1 code of the entries below on a
 * one-GPU machine; a peer missing for 120 s is an error, not a hang. */
int32_t osk_comm_init_loopback(int32_t device, int32_t rank, int32_t world, const uint8_t* id, int64_t slot_bytes,
                               osk_comm** out);
/* Testing build only: osk_comm_init_all's communicator (one process, local device i = rank i of n) whose
 * grouped all-gather is replaced by device copies, so devices may repeat — n local "devices" mapped to one
 * GPU run the multi-device code of osk_shards_search_merge on a one-GPU machine. */
int32_t osk_comm_init_all_loopback(const int32_t* devices, int32_t n, osk_comm** out);
/* Testing build only: runs the wide kernel's one-statement LDS-DMA helper (glds16_run, N = 1/2/4 DMAs at the
 * slab and bound-term strides) into out-of-order LDS destinations and counts the 16-B LDS words that differ from
 * the expected image (0 = every DMA landed exactly at its destination, nothing else written). */
int32_t osk_testing_glds_probe(int32_t device, int64_t* out_mismatches);

/* The whole multi-GPU query, host buffers, synchronous: every local view (views[i] on the
 * communicator's local device i) scans its shards, the per-shard top-k lists of every rank are
 * all-gathered once, and the coordinator reduce (from, size) runs on the device.  Every rank gets the
 * merged result.  shardIndex of a hit = the shard_index its view was created with (use the global
 * rank of the shard in sorted ShardId order).  accept: NULL or one host bitset pointer per segment
 * of every view, view 0's segments first.  Ranks may hold different numbers of shards (8 shards over 3
 * GPUs): the list slots per rank are agreed on every call (a small all-gather that overlaps the scans). */
int32_t osk_shards_search_merge(osk_comm* comm, osk_view* const* views, int32_t n_views, const void* queries,
                                int32_t n_queries, int32_t k, const uint64_t* const* accept, int32_t from,
                                int32_t size, float* out_scores, int32_t* out_docs, int32_t* out_shard_index,
                                int32_t* out_count, int64_t* out_total_hits, float* out_max_score);
/* The same for one GPU per process with device buffers, asynchronous on `stream`: d_queries
 * n_queries × dim on the view's device, d_accept as osk_view_search_device, shards_per_rank the
 * number of list slots per rank (≥ the view's shards; slots past them are empty), outputs as
 * osk_merge_device.  shards_per_rank should be the same on every rank (the caller knows the shard
 * layout, e.g. the largest shard count of any rank); at world > 1 the all-gather moves the communicator's
 * fixed block (osk_comm_set_device_limits), so a rank that differs gets count −1, never a hang.  A rank whose
 * own arguments are wrong (more shards in the view than shards_per_rank, k outside [1, OSK_MAX_K], a bad
 * from/size or batch) still issues that all-gather at world > 1, with a refusal header: every other rank's
 * reduce reports count −1 (communicator poisoned), and this rank returns OSK_ERR_INVALID without writing its
 * outputs.  Only null pointers and a view on another device return before the collective (a caller bug that
 * no shape can describe).  At world 1 every argument error returns at once. */
int32_t osk_shards_search_merge_device(osk_comm* comm, osk_view* view, const void* d_queries, int32_t n_queries,
                                       int32_t k, const uint64_t* const* d_accept, int32_t shards_per_rank,
                                       int32_t from, int32_t size, float* d_scores, int32_t* d_docs,
                                       int32_t* d_shard_out, int32_t* d_count, int64_t* d_total_hits,
                                       float* d_max_score, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* OSKNN_H */
