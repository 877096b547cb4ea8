// osk_filter.hip — filter pushdown by compaction: the accepted ordinals of every segment, in ascending
// order, packed into one array before the scan, so a selective filter costs a scan over the accepted
// rows only (one row-load round trip per 64 accepted rows) instead of a walk over every 64-row window
// of every tile (a load round trip per non-empty window).
//
// Lucene analogue: [L] AbstractKnnVectorQuery with a filter passes AcceptDocs = liveDocs ∩ filter bits
// to the reader, whose exact search visits only the accepted docs; OpenSearch's filter bitsets come
// from the BitsetFilterCache (S/index/cache/bitset/BitsetFilterCache.java:127-160).  Here the bitset is
// the C-ABI's accept bitset (⌈maxDoc/64⌉ u64 words, LSB-first) per segment; an absent bitset means
// every row of that segment is accepted.
//
//   filt_count   one wave per scan tile: accepted rows of the tile's row range  → tcnt[tile]
//   filt_scan    one workgroup: exclusive prefix of tcnt over the tile table → tpre[tile], and per
//                segment the accepted count scnt[seg] (a segment's tiles are contiguous in the table:
//                seg_tiles[seg] = [first, end))
//   filt_write   one wave per scan tile: its accepted ordinals, ascending, at
//                comp[seg_vrow[seg] + tpre[tile] − tpre[first tile of seg] + i]
// comp therefore holds, for segment g, scnt[g] ascending ordinals starting at its view row seg_vrow[g].
#include "osk_internal.h"
#include "osk_wave.h"

namespace osk {

namespace {

__device__ __forceinline__ bool accepted(const uint64_t* abits, const int32_t* o2d, int64_t row) {
    const int32_t doc = o2d ? o2d[row] : (int32_t)row;
    return (abits[doc >> 6] >> (doc & 63)) & 1ull;
}

// the accepted-row mask of the 64-row window starting at w0 (< we), dense field (doc == ord)
__device__ __forceinline__ uint64_t window_mask(const uint64_t* abits, int64_t w0, int64_t we) {
    const int64_t word = w0 >> 6;
    const int sh = (int)(w0 & 63);
    uint64_t m = abits[word] >> sh;
    if (sh && (word + 1) * 64 < we) m |= abits[word + 1] << (64 - sh);
    if (we - w0 < 64) m &= (1ull << (we - w0)) - 1ull;
    return m;
}

__global__ __launch_bounds__(64) void filt_count(FilterParams p) {
    const int lane = threadIdx.x;
    const TileDev t = p.tiles[blockIdx.x];
    const SegDev seg = p.segs[t.seg];
    const uint64_t* abits = p.accept[t.seg];
    int64_t n = 0;
    if (!abits) {
        n = lane == 0 ? t.row_end - t.row_begin : 0;   // summed over the wave below
    } else if (!seg.ord_to_doc) {
        // lane l takes windows l, l+64, … of the tile (one popcount each)
        for (int64_t w0 = t.row_begin + (int64_t)lane * 64; w0 < t.row_end; w0 += 64 * 64)
            n += __popcll(window_mask(abits, w0, t.row_end));
    } else {
        for (int64_t r = t.row_begin + lane; r < t.row_end; r += 64) n += accepted(abits, seg.ord_to_doc, r);
    }
    for (int o = 32; o >= 1; o >>= 1) n += __shfl_xor(n, o);
    if (lane == 0) p.tcnt[blockIdx.x] = (int32_t)n;
}

// exclusive prefix of tcnt[0, n_tiles] (tpre[n_tiles] = total) in chunks of 1024 with a carry
__global__ __launch_bounds__(1024) void filt_scan(FilterParams p) {
    __shared__ int32_t s_w[16];
    __shared__ int32_t s_carry;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) s_carry = 0;
    __syncthreads();
    for (int base = 0; base <= p.n_tiles; base += 1024) {
        const int i = base + tid;
        const int32_t v = i < p.n_tiles ? p.tcnt[i] : 0;
        int32_t x = v;   // inclusive wave scan
        for (int o = 1; o < 64; o <<= 1) {
            const int32_t y = __shfl_up(x, o);
            if (lane >= o) x += y;
        }
        if (lane == 63) s_w[wave] = x;
        __syncthreads();
        if (wave == 0) {
            int32_t w = lane < 16 ? s_w[lane] : 0;
            for (int o = 1; o < 16; o <<= 1) {
                const int32_t y = __shfl_up(w, o);
                if (lane >= o) w += y;
            }
            if (lane < 16) s_w[lane] = w;   // inclusive over waves
        }
        __syncthreads();
        const int32_t carry = s_carry;
        const int32_t excl = carry + (wave ? s_w[wave - 1] : 0) + x - v;
        if (i <= p.n_tiles) p.tpre[i] = excl;
        __syncthreads();
        if (tid == 1023) s_carry = excl + v;
        __syncthreads();
    }
    // per segment: accepted count = prefix at its tile end − prefix at its tile begin
    for (int g = tid; g < p.n_segs; g += 1024)
        p.scnt[g] = p.tpre[p.seg_tiles[g].y] - p.tpre[p.seg_tiles[g].x];
}

__global__ __launch_bounds__(64) void filt_write(FilterParams p) {
    const int lane = threadIdx.x;
    const TileDev t = p.tiles[blockIdx.x];
    const SegDev seg = p.segs[t.seg];
    const uint64_t* abits = p.accept[t.seg];
    uint32_t* out = p.comp + p.seg_vrow[t.seg] + (p.tpre[blockIdx.x] - p.tpre[p.seg_tiles[t.seg].x]);
    int64_t o = 0;
    for (int64_t w0 = t.row_begin; w0 < t.row_end; w0 += 64) {
        uint64_t m;
        if (!abits) {
            m = t.row_end - w0 >= 64 ? ~0ull : (1ull << (t.row_end - w0)) - 1ull;
        } else if (!seg.ord_to_doc) {
            m = window_mask(abits, w0, t.row_end);
        } else {
            m = __ballot(w0 + lane < t.row_end && accepted(abits, seg.ord_to_doc, w0 + lane));
        }
        if ((m >> lane) & 1ull) out[o + __popcll(m & ((1ull << lane) - 1ull))] = (uint32_t)(w0 + lane);
        o += __popcll(m);
    }
}

}  // namespace

hipError_t launch_filter_compact(const FilterParams& p, hipStream_t s) {
    if (p.n_tiles <= 0) return hipSuccess;
    hipLaunchKernelGGL(filt_count, dim3(p.n_tiles), dim3(64), 0, s, p);
    hipLaunchKernelGGL(filt_scan, dim3(1), dim3(1024), 0, s, p);
    hipLaunchKernelGGL(filt_write, dim3(p.n_tiles), dim3(64), 0, s, p);
    return hipGetLastError();
}

}  // namespace osk
