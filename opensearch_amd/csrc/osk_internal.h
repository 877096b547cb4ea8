// osk_internal.h — device-side structures and kernel launchers shared by osk_kernels.hip and
// osk_api.hip.  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <atomic>
#include "osk_common.h"

namespace osk {

// One segment as the scan kernels see it.
struct SegDev {
    const void* rows;            // f32: float4[n_rows][units]; byte: 16-B chunks [n_rows][units]
    const float* xnorm_f;        // f32 COSINE: |x|² per row (lane-layout order), else null
    const int32_t* xnorm_i;      // byte: Σx² per row (exact), else null
    const int32_t* ord_to_doc;   // null = dense (doc == ord)
    int64_t n_rows;
    int32_t doc_base;            // LeafReaderContext.docBase inside the shard
    int32_t shard;               // result group
};

// A contiguous run of rows of one segment, scanned by one 256-thread workgroup.
struct TileDev {
    int32_t seg;
    int32_t shard;
    int64_t row_begin;
    int64_t row_end;
};

struct ScanParams {
    const SegDev* segs;
    const TileDev* tiles;
    const uint64_t* const* accept;   // device array [n_segs] of bitsets (entries may be null), or null
    const void* q;                   // this launch's queries, each padded to L*V units (zeros)
    const float* qnorm_f;            // this launch's query norms (COSINE f32)
    const int32_t* qnorm_i;          // this launch's query Σq² (byte)
    uint64_t* cand;                  // [nq_total][n_tiles][k] per-tile candidate keys
    unsigned long long* visited;     // [n_segs] or null (counted by the q0 == 0 launch only)
    int n_tiles;
    int q0;                          // global index of this launch's first query
    int q_count;                     // queries in this launch (≤ NQ of the instantiation)
    int units;                       // float4s (f32) / 16-B chunks (byte) per stored row
    int k;
    int sim;
    int dim;
};

constexpr int kBlock = 256;          // 4 wavefronts per workgroup
constexpr int kMaxNQ = 8;            // queries per streaming-scan launch
constexpr int kScanMaxK = 64;        // k the streaming scans' wave lists hold (beyond: the select path)
constexpr int kKsAlign = 4;        // MFMA K-steps (32 dims) per segment split copy: a multiple of this
constexpr int kKC = 16;              // candidates per (query, shard) of the batched MFMA path (k ≤ kKC − 4)

// ---- batched MFMA path (osk_mfma.hip) ----
struct MfmaUnit {            // a run of 128-row tiles of one segment, one workgroup
    int32_t seg;
    int32_t shard;
    int64_t tile_begin;      // in 128-row tiles of the segment
    int64_t tile_end;
    int64_t vrow_base;       // view-global row index of the segment's ord 0
};

struct MfmaParams {
    const SegDev* segs;
    const MfmaUnit* units;
    const void* const* seg_split;     // per segment: fragment-ordered bf16 hi/lo copy
    const float* const* xsqrt;        // per segment: |x| per row
    const uint64_t* const* accept;
    const void* qsplit;               // queries in the same fragment order
    const float* qnorm;               // per query |q|² (approx transforms)
    uint64_t* cand;                   // [nq][n_units*2][kKC] approx candidate keys (doc = view row)
    unsigned long long* visited;
    const uint64_t* thr_keys;         // pilot: [nq][n_shards][kKC] merged keys (main pass), or null
    const int32_t* thr_counts;        // pilot: [nq][n_shards]
    int n_shards;
    int n_units;
    int KS;                           // 32-dim K-steps
    int nq;
    int nq_pad;
    int ablate;
    int sim;
    unsigned long long* full_tiles;   // tiles whose epilogue took the staging path (counter "mfma_full_tiles")
};

struct RescoreParams {
    const SegDev* segs;
    const int64_t* seg_vrow_begin;    // view row of each segment's ord 0 (ascending)
    const uint64_t* akeys;            // [nq][n_shards][kKC] merged approx candidates
    const void* q;                    // padded fp32 queries ([nq][L·V] float4)
    const float* qnorm_dev;           // |q|² in the device lane order (COSINE) or null
    const float* qnorm_approx;        // |q|² (any order) for the bound
    const float* shard_maxnorm2;      // max |x|² per shard
    uint64_t* shard_keys;             // [nq][n_shards][k]
    int32_t* shard_counts;
    int* flags;                       // [nq] set when a certificate fails
    double c;                         // error-bound constant
    int n_shards;
    int n_segs;
    int units;
    int k;
    int sim;
};

hipError_t launch_split_rows(const float4* rows, int64_t n_rows, int units, int KS, int64_t n_rb,
                             void* out, hipStream_t s);
hipError_t launch_row_sqrt(const float* xn, int64_t n, float* out, hipStream_t s);
hipError_t launch_max_norm2(const float* xn, int64_t n, unsigned* out, hipStream_t s);
hipError_t launch_mfma_cand(const MfmaParams& p, int n_qblocks, bool pilot, hipStream_t s);
hipError_t launch_rescore(int cfg, int nq, const RescoreParams& p, hipStream_t s);

// ---- certified int8 prefilter (osk_sq8.hip) ----
// A float32 segment keeps an int8 copy (per-row symmetric scale) and per-row bound terms.  The
// prefilter scan streams the int8 copy (¼ of the bytes), bounds every row's device-order fp32 score
// from above and below, and keeps per tile the kKQ rows with the highest upper bound; the settle
// kernel re-scores exactly the rows that can still reach the shard's top k and proves the rest
// cannot.  Results are bit-identical to the fp32 streaming scan.
constexpr int kKQ = 16;              // per-tile candidate list of the prefilter (k ≤ kKQ)
constexpr int kSliceLists = 32;      // wave lists per settle workgroup (32 × kKQ = 512 entries)
constexpr int kLGroupLists = 4096;   // lists whose best lower bounds define one settle threshold

struct Sq8Params {
    const SegDev* segs;
    const TileDev* tiles;
    const uint64_t* const* accept;
    const int4* const* rows8;        // per segment: int8 rows [n_rows][units8] 16-B units
    const float4* const* aux;        // per segment: {scale, scale·|q8|, |x − scale·q8|, |x|²} per row
    const int64_t* seg_vrow;         // view row of each segment's ord 0
    const int4* q8;                  // this launch's int8 queries [NQ][units8]
    const float4* qc;                // per query {scale, |b − s·q8|, s·|q8| + |b − s·q8|, |b|²}
    const float* qn_dev;             // this launch's |q|² in the device lane order (COSINE)
    uint64_t* cand;                  // [nq][n_lists][kKQ] keys (upper-bound score, view row); list = tile·4 + wave
    uint32_t* cand_lb;               // [nq][n_lists][kKQ] sortable lower-bound scores
    uint32_t* list_lbmax;            // [nq][n_lists] best lower bound of each list (0 = empty)
    unsigned long long* visited;
    int n_tiles;
    int n_lists;                     // 4 · n_tiles
    int q0;
    int q_count;
    int units8;
    int sim;
    float gam;                       // fp32 dot rounding: |dot_dev − x·b| ≤ gam·(|x|² + |b|²)
    float g2;                        // fp32 d² rounding:  |d²_dev − d²| ≤ g2·d²
    float cos_slack;                 // COSINE quick test: norm-order slack
    // sq8_mfma only.  pilot = 1: each wave scores just its first 16 (accepted) rows; the tile's top k
    // lower-bound keys per query go to pilot_keys [q_count][n_tiles][k]; merged per (query, shard)
    // into thr_keys [q_count][n_shards][k] / thr_counts.  pilot = 0: the k-th best sampled
    // lower bound T of the (query, shard) is a floor under every wave list's quick threshold: a row
    // with ub < T ≤ the shard's k-th best lower bound scores below the shard's k-th exact score.
    int pilot;
    const int4* const* rows8t;       // sq8_mfma: per segment, the tiled int8 copy (launch_sq8_tile)
    int nt;                          // sq8_mfma: non-temporal row loads (A/B knob sq8_mfma_nt)
    int ablate;                      // A/B timing only (results wrong): 1 skip the epilogue, 2 skip the MFMAs
    int ring_slots;                  // sq8_mfma: > 1 = LDS-DMA ring of this many 16-row groups per wave
                                     // (unfiltered, ≤ 256 dims; tune sq8_mfma_ring), 0 = register loads
    int k;
    int n_shards;
    uint64_t* pilot_keys;
    const uint64_t* thr_keys;
    const int32_t* thr_counts;
    // gather mode (filtered sq8_scan, osk_filter.hip compaction): the grid runs over gather tiles
    // {seg, shard, j, nj} — tile j of nj over segment seg's scnt[seg] accepted ordinals at
    // comp[seg_vrow[seg] …] — instead of `tiles`; null = the row-range tiles
    const int4* gtiles;
    const uint32_t* comp;
    const int32_t* scnt;
    int gather_min;                  // at most one gather tile per this many accepted rows of a segment
    // sq6_scan (osk_sq6.hip): per segment, the 6-bit tiled codes and their bound terms; the query's nibble
    // split ([8C half-chunks][bh 4 dwords, bl 4 dwords]) and its 6-bit bound terms; the per-(query, shard)
    // floor buckets [q][n_shards][kFloorBuckets] (sortable lower bounds; rows8 / aux / q8 / qc are the
    // int8 re-bound of the rows that pass the 6-bit test)
    const void* const* rows6;
    const float4* const* aux6;
    const int4* q6;
    const float4* qc6;
    uint32_t* floor;
    unsigned long long* counters;    // sq6_scan adds its int8 re-bounds to [3] (SettleParams::counters)
    unsigned long long* seg_rebound; // calibration probes: the int8 re-bounds per segment [n_segs], or null
    const int32_t* tile_order;       // sq6_scan: the tile of each workgroup (tiles interleaved over shards)
    uint2* cand6;                    // sq6_scan → sq6_rebound: per list, the rows that passed the 6-bit test
                                     // {row, its 6-bit test value (osk_sq6.hip cand6_value)}
    int32_t* cnt6;                   // [q][n_lists] their count (> cap6: overflowed)
    int cap6;
    const float4* const* auxt;       // sq8_wide: per segment, the 16-row groups' bound terms (launch_sq8w_build)
    int wide_grid;                   // sq8_wide: persistent workgroups (the device's CUs)
    int n_segs;                      // sq6_rebound: the view's segments (LDS per-segment counts when ≤ 64)
    int rb_stride;                   // sq6_rebound: 1 = wave gw takes lists gw, gw + W, … (tune sq6_rebound_stride)
    int rb_wg_per_cu;                // sq6_rebound: workgroups per CU (0 = as many as fit; tune sq6_rebound_wgs)
    int rb_retest;                   // sq6_rebound: re-test candidates at the 6-bit level against the final floor
    int quarter_begin, quarter_end;  // sq8_wide: the launch's quarters in tile order (end 0: all)
    int pilot_rows;                  // sq8_wide pilot: rows bounded per quarter (0 = kWidePilotRows)
    int wide_defer;                  // sq8_wide: defer insertions to the quarter's end when LDS allows (tune)
    int wide_qcap;                   // (set by launch_sq8_wide: entries per wave's deferred queue, 0 = immediate)
    const uint32_t* floors;          // sq8_wide: [q_count][n_shards] floor score (sortable bits; 0 = none)
    const float4* quarter_bm;        // sq8_wide: [4·n_tiles] the quarters' row maxima (launch_wide_quarter_max)
    const void* wide_qtable;         // sq8_wide: [4·n_tiles] the quarters' descriptors in tile order (null: computed)
    int wide_claim;                  // sq8_wide_rows: waves claim groups from a per-quarter counter (0: fixed interleave)
};

struct SettleParams {
    const SegDev* segs;
    const int64_t* seg_vrow;
    const uint64_t* cand;            // the scan's wave lists [nq][n_lists][kKQ]
    const uint32_t* cand_lb;
    const uint32_t* list_lbmax;      // [nq][n_lists]
    const void* q;                   // padded fp32 queries [nq][UP] float4
    const float* qnorm;              // |q|² device order (COSINE)
    uint64_t* shard_keys;            // [nq][n_shards][k]
    int32_t* shard_counts;
    int* flags;                      // [nq] set when some list of the query was re-scanned exactly
    unsigned long long* counters;    // [0] queries with an exactly re-scanned list, [1] rows re-scored,
                                     // [2] lists re-scanned exactly
    const int4* slices;              // [n_slices] {list_begin, list_end, L-group begin, L-group end}
    const int32_t* shard_slice_begin;// [n_shards + 1]
    const TileDev* tiles;            // the view's tiles (exact re-scan of an overflowed list)
    const uint64_t* const* accept;   // per-segment accept bitsets (or null)
    uint64_t* part;                  // [nq][n_slices][k] per-slice exact top k
    int n_slices;
    int n_lists;                     // 4 · n_tiles (list = tile·4 + scan wave)
    int scan_R;                      // rows per wave-iteration of the int8 scan (its per-wave row split)
    int n_shards;
    int n_segs;
    int units;
    int k;
    int sim;
    int force_fail;                  // tests: re-scan every list exactly
    const int4* gtiles;              // gather mode (see Sq8Params): lists are gather tile·4 + wave
    const uint32_t* comp;
    const int32_t* scnt;
    int gather_min;
    unsigned long long* trace;       // A/B only: per (query, slice) 8 slots of phase timestamps, or null
    const int32_t* shard_tile_begin; // sq8_settle_wide: [n_shards + 1] (a shard's lists are 4·[begin, end))
};
// The settle of wide batches (osk_sq8.hip): one workgroup per (shard, query) over all the shard's lists —
// the per-slice settle's ≈ n_lists / 32 workgroups per query left 786k workgroups at 100M rows × 1024
// queries (4.3 ms, mostly threshold loads).  Unfiltered views only; writes shard_keys / shard_counts itself.
hipError_t launch_sq8_settle_wide(int cfg, int nq, const SettleParams& p, hipStream_t s);

// Filter pushdown by compaction (osk_filter.hip): per segment, the accepted ordinals in ascending order
// at comp[seg_vrow[seg] …], scnt[seg] of them.
struct FilterParams {
    const SegDev* segs;
    const TileDev* tiles;               // the view's scan tiles (row ranges of one segment each)
    const uint64_t* const* accept;      // per segment: accept bitset or null (= every row accepted)
    const int64_t* seg_vrow;            // view row of each segment's ord 0
    const int2* seg_tiles;              // per segment: [first tile, end tile) in the tile table
    int32_t* tcnt;                      // [n_tiles] accepted rows per tile
    int32_t* scnt;                      // [n_segs] accepted rows per segment
    uint32_t* comp;                     // [view rows] compacted ordinals
    int n_tiles;
    int n_segs;
};
hipError_t launch_filter_compact(const FilterParams& p, hipStream_t s);

// ---- the select path: exact top-k for any k ≤ OSK_MAX_K (osk_select.hip) ----
constexpr int kSelCap = 16384;       // candidates per (query, shard) the select path sorts in LDS
constexpr int kSelDigit = 11;        // radix select digit width (2048-bin histograms)
constexpr int kSelBins = 1 << kSelDigit;
constexpr int kSelShift0 = 32 - kSelDigit;   // the first digit of a 32-bit LB
// Global per-shard histograms are kept in kSelRep replicas (a tile adds into replica tile % kSelRep):
// every tile of a shard adding into the same few bins serialised on those addresses (≈30 ns per
// same-address device atomic: 40 µs per pass at C3)
constexpr int kSelRep = 16;
struct RadixState {
    uint64_t prefix;                 // the digits of the k-th largest value decided so far
    int32_t krem;                    // its rank among the values that share them
    int32_t all;                     // ≤ k accepted rows: take every one
    int32_t pad;
};
struct SelParams {
    const SegDev* segs;
    const TileDev* tiles;
    const int64_t* seg_vrow;
    const int32_t* shard_tile_begin; // [n_shards + 1]: a shard's tiles are contiguous
    const int32_t* tile_coff;        // [n_tiles]: the tile's first row's slot in its shard's candidate region
    const uint64_t* const* accept;
    unsigned long long* visited;     // [n_segs] or null
    int n_tiles, n_shards, n_segs;
    int k, sim, dim, units, units8, enc;
    int exact;                       // 1: 64-bit keys of exact scores; 0: int8 bounds LB/UB + exact re-score
    int writer;                      // bounds writer variant (tune sel_writer)
    const void* q;                   // this query, padded (fp32 UP float4 / int8 16-B units)
    const float* qnorm;              // its |q|² in the device lane order (COSINE)
    const int4* q8;                  // bounds mode: its int8 copy and bound terms
    const float4* qc;
    const int4* const* rows8;
    const float4* const* aux;
    float gam, g2;
    uint32_t* lb;                    // bounds mode, [view rows]
    uint32_t* ub;
    uint64_t* keys;                  // exact mode, [view rows]
    RadixState* state;               // [n_shards]
    uint32_t* hist;                  // [n_shards][kSelRep][kSelBins]
    uint64_t* cand;                  // [n_shards][cap]: tile t's candidates at tile_coff[t] (no atomics)
    uint64_t* cand2;                 // [n_shards][cap]: a shard's candidates packed (only past kSelCap)
    int32_t* tile_count;             // [n_tiles]: candidates per tile
    int cap;                         // the largest shard's rows: a shard's candidates always fit
    uint64_t* out_keys;              // this query's [n_shards][k]
    int32_t* out_counts;             // [n_shards]
};
// one query: writer → radix select → collect → (re-score) → sort; cfg = the view's fp32/byte lane cfg
hipError_t launch_select_one(const SelParams& p, int cfg, hipStream_t s, hipEvent_t ev_start = nullptr,
                             hipEvent_t ev_stop = nullptr);
// Layout of a gathered multi-rank image (osk_comm.hip).  Default: rank r's lists [nq][sl][k] at
// r·nq·sl·k words, shardIndex of slot (r, j) at shard_index[r·sl + j], no header.  The exchange gathers
// one block per rank instead — [keys nq·sl·k][header kXHdrWords][shard indices sl int32] — so every
// call carries its own shardIndex and a header that the reduce compares across ranks: a rank whose
// header differs (another call sequence number, batch, k, from/size, shards per rank or query
// fingerprint) makes every query's count −1 and records the mismatch in `err` (host memory).
constexpr int kXHdrWords = 8;
constexpr uint64_t kXMagic = 0x4F534B5800000001ull;     // header word 0 of a block: "OSKX", format 1
constexpr uint64_t kXRefused = 0x4F534B58FFFFFFFFull;   // ...of a rank that refused its call (device limits)
struct XHdrWords {
    uint64_t w[kXHdrWords];
};
struct XLayout {
    size_t rank_words = 0;            // u64 words per rank block (0 = nq·sl·k, no header)
    int si_stride = 0;                // int32 between ranks' shard index arrays (0 = sl)
    const uint64_t* hdr = nullptr;    // rank 0's header (rank r's at hdr + r·rank_words); null = none
    int64_t* err = nullptr;           // [flag, rank-0 seq, first mismatching rank, its seq]
};
// The coordinator reduce: merge_coord (one workgroup per query, ≤ kCoordMax = 4096 hits ranked in LDS)
// or, for more hits per query, merge_rank (launch_merge_rank); same layout, same outputs.
hipError_t launch_coord_reduce(const uint64_t* shard_keys, const int32_t* shard_counts, const int32_t* shard_index,
                               int nq, int n_ranks, int sl, int k, int from, int size, float* scores, int32_t* docs,
                               int32_t* shard_out, int32_t* count, int64_t* total_hits, float* max_score,
                               hipStream_t s, const XLayout& x = XLayout{});
// coordinator reduce for lists of any length (merge_coord's layout and outputs; no 4096-hit limit)
hipError_t launch_merge_rank(const uint64_t* keys, const int32_t* counts, const int32_t* shard_index, int nq,
                             int n_ranks, int sl, int k, int from, int size, float* scores, int32_t* docs,
                             int32_t* shard_out, int32_t* count, int64_t* total_hits, float* max_score,
                             hipStream_t s, const XLayout& x = XLayout{});
// The exchange block's trailer of this rank: header words w[0..kXHdrWords) with w[5] replaced by a
// fingerprint of the query bytes, then the shard indices (sl slots: the view's n_shards, pads INT32_MAX).
hipError_t launch_xhdr_fill(uint64_t* hdr, const uint64_t* w, const void* queries, int64_t query_bytes,
                            const int32_t* shard_index, int n_shards, int sl, hipStream_t s);

hipError_t launch_sq8_quantize(const float4* x, int64_t n, int units, int pitch, int units8, void* out8,
                               float4* aux, int mode, hipStream_t s);
// ev_start / ev_stop (optional): stamped by the kernel's own dispatch packet (hipExtLaunchKernelGGL),
// so timing a launch adds no marker packets (and no gaps) to the stream
hipError_t launch_sq8_scan(int nq, const Sq8Params& p, hipStream_t s, hipEvent_t ev_start = nullptr,
                           hipEvent_t ev_stop = nullptr);
int sq8_lanes(int units8);         // lanes per row of the int8 scan
// int8 MFMA prefilter scan: ≤ kMfmaQueries queries per launch, rows ≤ 1024 int8 dims (sq8_mfma_supported)
constexpr int kMfmaQueries = 32;
constexpr int kMfmaScanR = 16;      // its rows per wave-iteration (the settle's scan_R)
int sq8_mfma_supported(int units8);
int sq8_mfma_ks(int units8);
int sq8_ring_slots(int units8, int qb, int want);   // sq8_mfma LDS-DMA ring depth (0 = register loads)        // its 64-dim k-steps per row for this row width
// row-major int8 rows → blocks of 16 rows × ks slabs of 1 KiB (row r of a block at r·64 B; zero past
// the last row and past units8)
hipError_t launch_sq8_tile(const void* q8, int64_t n_rows, int units8, int ks, void* out, hipStream_t s);
hipError_t launch_sq8_mfma(const Sq8Params& p, hipStream_t s, hipEvent_t ev_start = nullptr,
                           hipEvent_t ev_stop = nullptr);
// int8 MFMA prefilter for large batches (osk_sq8w.hip): kWideQ queries per launch, 32 per wave, rows
// ≤ 768 int8 dims, unfiltered.  Persistent: one workgroup of 8 waves per CU streams its share of the
// (tile, quarter) row ranges — the settle's list of a scan wave with scan_R = kMfmaScanR — through an
// LDS-DMA ring once; every wave scores its 32 queries against every staged row (lists per (quarter, query)
// in LDS).  It reads its own copy of the rows (launch_sq8w_build).  pilot = 1: each quarter's first step only,
// and per query the best lower-bound key of it to pilot_keys [q][4·n_tiles].
constexpr int kWideQB = 2;                      // 16-query MFMA blocks per wave
constexpr int kWideWaves = 8;                   // two per SIMD
constexpr int kWideQ = kWideWaves * 16 * kWideQB;   // queries per launch
constexpr int kWidePilotRowsDefault = 128;   // the wide pilot's rows per quarter (≥ 512 dims: 256)...
constexpr int kWidePilotSample = 65536;      // ...raised to sample at least this many rows per shard (≤ 1,024 a quarter)
constexpr int kAuxGroupF4 = 22;                 // float4 per 16-row group of the tiled bound terms
int sq8_wide_supported(int units8);
int sq8_wide_ks(int units8);                    // its 64-dim slabs per row: 2, 4, 8 or 12
hipError_t launch_sq8_wide(const Sq8Params& p, hipStream_t s, hipEvent_t ev_start = nullptr, hipEvent_t ev_stop = nullptr);
// the wide kernel's main passes for ≤ 128-dim rows without a step barrier (osk_sq8w.hip sq8_wide_rows)
bool sq8_wide_rows_supported(int u8);
hipError_t launch_sq8_wide_rows(const Sq8Params& p, hipStream_t s, hipEvent_t ev_start = nullptr,
                                hipEvent_t ev_stop = nullptr);
#ifdef OSK_TESTING
hipError_t launch_glds_probe(const int4* src, int4* out, hipStream_t s);   // (osk_testing_glds_probe)
#endif
// The wide kernel's copy of a segment's fp32 rows (units float4 per row): int8 codes with ONE scale per
// 16-row group (s_g = the group's max |x| / 127), in the MFMA-tiled layout (16-row blocks × sq8_wide_ks slabs of
// 1 KiB, chunk-major), and per group kAuxGroupF4 float4 of bound terms (352 B): s_g[16] (COSINE: each row's
// quick-test factor s_g / √|x|² instead), (s_g|q_x|)[16], |δ_x|[16],
// |x|²[16] (struct of arrays: a lane reads its 4 rows' terms in one ds_read_b128), {max s|q|, max |δ|, max |x|²,
// min |x|²}, {s_g, f_cos, zero-row flag, 0} (the quick test's per-group factor) and (COSINE) the rows' device-order
// |x|² (xnorm; zeros without).  Rows past the last: zero codes and terms, not in the extrema.  The kernel stages
// the first 18 float4 (COSINE all 22) with the rows.
hipError_t launch_sq8w_build(const float4* rows, int64_t n_rows, int units, int units8, const float* xnorm, int cosine,
                             void* codes, float4* auxt, hipStream_t s);
// Per (tile, quarter) of a view: {max s|q|, max |δ|, max |x|², min |x|²} over its rows (the wide kernel's
// quick-test terms, from the tiled bound terms' group maxima), out [4·n_tiles]
hipError_t launch_wide_quarter_max(const TileDev* tiles, int n_tiles, const float4* const* auxt, float4* out,
                                   hipStream_t s);
// The wide kernel's per-(query, shard) floors [nq][n_shards]: base (or 0), raised to the k-th best of the
// shard's pilot keys (pilot_keys [nq][n_lists], one per quarter) or of its lists' maximum lower bounds
// (list_lbmax [nq][n_lists]; 0 = not written); the shard's quarters / lists are [shard_list_begin[s], [s + 1]).
// Sortable score bits; a floor at or below score 0 is dropped (ties at the clamp).
hipError_t launch_wide_quarter_table(const TileDev* tiles, const int32_t* tile_order, int n_q, int ks,
                                     const void* rows8t, const void* auxt, const int64_t* seg_vrow,
                                     const float4* quarter_bm, void* out, hipStream_t s);
hipError_t launch_wide_floor(const uint32_t* list_lbmax, const uint64_t* pilot_keys, int n_lists,
                             const int32_t* shard_list_begin, int n_shards, int nq, int k, const uint32_t* base,
                             uint32_t* floors, hipStream_t s);
// The 6-bit tier's share of the query prep (C = 0: none): the nibble-split query [nq_pad][64·C dwords],
// its bound terms, and the floor buckets [nq_pad][floor_n] zeroed
struct Sq6Prep {
    uint32_t* q6 = nullptr;
    float4* qc6 = nullptr;
    uint32_t* floor = nullptr;
    int floor_n = 0;
    int C = 0;
};
hipError_t launch_sq8_prep(int cfg, const float* src, int dim, int nq, int nq_pad, int UP, int units8, float4* qpad,
                           float* qnorm, void* q8, float4* qc, int* flags, hipStream_t s, const Sq6Prep& q6 = Sq6Prep{});
// ---- the 6-bit first tier (osk_sq6.hip): single unfiltered queries over float32 rows of ≥ 512 dims ----
int sq6_chunks(int dim);                 // C: half-chunks of 32 dims per lane (8 lanes per row)
int sq6_supported(int dim);
int64_t sq6_bytes(int64_t n_rows, int dim);   // the tiled codes + bound terms of a segment
constexpr int kSq6ScanR = 8;             // rows per wave-iteration of sq6_scan (the settle's scan_R)
constexpr int kFloorBuckets = 64;       // sq6_scan's floor: the k-th best of 64 bucket maxima of lists' best lbs,
constexpr int kFloorStride = 16;        // one 64-B line per bucket (uint32 units)
constexpr int kSq6Probes = 4;            // calibration probes of the 6-bit tier per segment (osk_seg::sq6_state)
constexpr int kSq6Cap = 256;             // candidate rows per list between the 6-bit pass and the int8 re-bound
hipError_t launch_sq6_quantize(const float4* x, int64_t n, int units, int dim, void* out, float4* aux, hipStream_t s);
hipError_t launch_sq6_scan(const Sq8Params& p, int dim, hipStream_t s, hipEvent_t ev_start = nullptr,
                           hipEvent_t ev_stop = nullptr);
hipError_t launch_sq8_settle(int cfg, int nq, const SettleParams& p, hipStream_t s);

int cfg_index(int units);

// Process-wide tuning knobs (osk_tune_set).  Every field is an atomic int: a search reads each knob
// once where it decides on it, and a concurrent osk_tune_set can only switch between valid settings
// (every path returns the same exact results).  The fields marked TESTING are settable only in the
// testing build (libosknn_testing.so, -DOSK_TESTING): they corrupt results or trace internals.
struct Tuning {
    std::atomic<int> host_batching{1};       // host entries batch concurrent unfiltered calls (osk_api.hip batched_call)...
    std::atomic<int> host_batch_leaders{1};  // ...with at most this many batches in flight per view (1: measured best)
    std::atomic<int> scan_nt{1};          // non-temporal corpus loads in scan_f32 (+4% HBM rate, profiles/r01_scan_ab.txt)
    std::atomic<int> tiles_target{0};     // workgroup tiles per view (scan grid size); 0 = whole rounds of the chip's
                              // resident slots (osk_view_create)
    std::atomic<int> tile_slots_per_cu{4};    // resident scan workgroups per CU (4 waves/SIMD, 256-thread groups)
    std::atomic<int> tile_large_slots{24};    // views of ≥ CUs × this × tile_min_rows rows: CUs × this tiles (0 = off)
    std::atomic<int> tile_large_slots_512{12};   // …the same for views of ≥ 512-dim rows
    std::atomic<int> tile_max_rounds{4};      // at most this many rounds (10M rows: 4096 tiles, profiles/r01e)
    std::atomic<int> tile_min_rows{1024}; // ...and at least this many rows per tile (1.25M rows: 1024 tiles of 1221
                              // rows, 4360 QPS vs 3968 for 4096 tiles of 305 rows — profiles/r01e/tiles_ab.txt)
    std::atomic<int> mfma_min_batch{96};  // batches ≥ this may take the bf16×3 MFMA candidate path (0 = never)...
    std::atomic<int> sq8_cost_pct{100};   // ...when its blocks cost no more than the int8 prefilter's launches (a
                              // per-row cost model of both, view_search_device), the prefilter's side scaled
                              // by this / 100; else the int8 prefilter
    std::atomic<int> mfma_units{0};       // workgroup units of the MFMA candidate pass per view (0: auto)
    std::atomic<int> sq8{1};              // certified int8 prefilter for float32 batches below mfma_min_batch
    std::atomic<int> sq6{1};              // ...whose single unfiltered queries scan the 6-bit tier where the dim has one,
    std::atomic<int> sq6_probe_pct{10};   // ...unless its first probes re-bound more than this % of a segment's rows
    std::atomic<int> gather_min{0};       // ...at most one gather tile per this many accepted rows (0 = every gather
                                          // tile; fewer, longer tiles were slower: profiles/r02c/gather_min_ab.jsonl)
    std::atomic<int> sel_writer{2};       // select path bounds writer: 0 U4 + Java transform, 1 U4 fast COSINE
                                          // bounds, 2 U2 fast, 3 U1 fast (same results; speed only)
    std::atomic<int> select_mid_k{1};     // float32 12 < k ≤ 64 with the prefilter on: the select path's int8
                                          // bounds pass instead of the fp32 streaming scan (0 = the scan)
    std::atomic<int> filter_gather{1};    // filtered prefilter scans (VALU sq8_scan) compact the accepted ordinals
                                          // first and scan them (osk_filter.hip); 0 = walk the bitset windows
    std::atomic<int> sq8_mfma_nt{1};      // A/B: non-temporal row loads in sq8_mfma
    std::atomic<int> i8_stream{1};        // byte fields, one query, no filter: scan_i8_stream (0 = scan_i8)
    std::atomic<int> call_timing{0};      // host entries time each call on the device (osk_last_call_device_ns)
    std::atomic<int> sq8_mfma_ring{-1};   // sq8_mfma LDS-DMA ring slots per wave (≤ 256 dims, unfiltered):
                                          // -1 = as many as fit 2 workgroups per CU, 0 = off (register loads)
    std::atomic<int> sq8_mfma_queries{32};    // queries per sq8_mfma launch: 16 or 32 (two MFMA chains per row operand)
    std::atomic<int> sq8_mfma_ablate{0};  // TESTING. A/B timing only: 1 skip sq8_mfma's epilogue, 2 its MFMAs (results wrong)
    std::atomic<int> sq8_mfma_min{2};     // prefilter batches ≥ this scan on int8 MFMA, 16 queries per launch (0 = never)
    std::atomic<int> sq8_wide_min{64};    // ...and unfiltered batches ≥ this on the wide kernel, kWideQ per launch, when
                                          // its cost model beats sq8_mfma's (0 = never)
    std::atomic<int> sq8_wide_grid{0};    // wide kernel's persistent workgroups (0 = one per CU)
    std::atomic<int> sq8_wide_pilot_rows{0};   // wide pilot rows per quarter (0 = 128, 256 at ≥ 512 dims)
    std::atomic<int> sq6_rebound_retest{1};   // sq6_rebound: the final-floor 6-bit re-test (0: gather every candidate)
    std::atomic<int> sq6_rebound_stride{1};   // sq6_rebound: strided list assignment (0: contiguous)
    std::atomic<int> sq6_rebound_wgs{0};      // sq6_rebound: workgroups per CU (0: as many as fit)
    std::atomic<int> sq8_wide_rows{1};    // wide kernel, ≤ 128 dims: the main passes on sq8_wide_rows (0: sq8_wide)
    std::atomic<int> sq8_wide_rows_claim{1};   // sq8_wide_rows: dynamic group claims per quarter (0: wave + 8i)
    std::atomic<int> sq8_scan_deep{0};    // single-query sq8_scan ≤ 256 dims: U = 8 row groups in flight per wave
    std::atomic<int> sq8_wide_rows_qcap{0};   // (tests) its deferred queue per owner wave, entries (0: kRowsQC)
    std::atomic<int> sq8_wide_defer{1};   // wide kernel: defer list insertions to each quarter's end (0: immediate)
    std::atomic<int> sq8_wide_quarter_rows{0};   // rows per wide quarter, read when a view builds its table (0 = auto)
    std::atomic<int> sq8_wide_force{0};   // (tests) the wide kernel for every eligible batch, whatever the model says
    std::atomic<int> sq8_wide_phase{8};   // the wide kernel's first pass covers 1/this of the quarters, whose lists
                                          // raise the floors of the rest (0: one pass)
    std::atomic<int> sq8_force_fallback{0};   // TESTING. tests: every list of a prefiltered search is re-scanned exactly
    std::atomic<int> settle_trace{0};     // TESTING. A/B only: record settle phase timestamps (debug copy "settle_trace")
    std::atomic<int> mfma_ablate{0};      // TESTING. A/B only: 1 skip the epilogue, 2 skip query staging, 4 skip corpus staging,
                              // 8 force the full staging epilogue, 16 skip the pilot pass, 32 skip the
                              // main epilogue's quick tests, 64 skip its merge (barriers + list inserts)
                              // (results are wrong and the exact fallback is skipped)
};
extern Tuning g_tuning;

hipError_t launch_scan(int enc, int cfg, int nq, const ScanParams& p, hipStream_t s, hipEvent_t ev_start = nullptr,
                       hipEvent_t ev_stop = nullptr);
hipError_t launch_row_norms_f32(const float4* rows, int64_t n_rows, int units, int cfg,
                                float* out, hipStream_t s);
hipError_t launch_row_norms_i8(const int4* rows, int64_t n_rows, int units, int32_t* out,
                               hipStream_t s);
hipError_t launch_synth(void* rows, int64_t n_rows, int dim, int units, int enc, uint64_t seed,
                        int dist, int64_t row0, hipStream_t s);
hipError_t launch_prep_queries(const void* src, int64_t row_bytes, int nq, void* dst, int units, int nq_pad,
                               hipStream_t s);
hipError_t launch_pad_rows(const void* src, int64_t src_pitch, void* dst, int64_t dst_pitch,
                           int64_t n_rows, int64_t row_bytes, hipStream_t s);
hipError_t launch_merge_shards(const uint64_t* cand, int n_tiles, const int32_t* shard_tile_begin,
                               int n_shards, int nq, int k, uint64_t* shard_keys,
                               int32_t* shard_counts, hipStream_t s, int kin = 0);   // kin: keys per tile (0 = k)
hipError_t launch_merge_coord(const uint64_t* shard_keys, const int32_t* shard_counts,
                              const int32_t* shard_index, int nq, int n_ranks, int sl, int k, int from,
                              int size, float* scores, int32_t* docs, int32_t* shard_out,
                              int32_t* count, int64_t* total_hits, float* max_score,
                              hipStream_t s, const XLayout& x = XLayout{});

}  // namespace osk
