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
//   filt_write   one wave per scan tile: its offset in the segment's list (Σ tcnt of the segment's
//                earlier tiles; a segment's tiles are contiguous in the table, seg_tiles[seg] =
//                [first, end)), then its accepted ordinals, ascending, at comp[seg_vrow[seg] + offset + i];
//                the segment's last tile writes the segment's count scnt[seg]
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

// one wave per tile, 4 tiles per workgroup (6k one-wave workgroups dispatch slower than 1.5k of four)
__global__ __launch_bounds__(256) void filt_count(FilterParams p) {
    const int lane = threadIdx.x & 63;
    const int tile = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (tile >= p.n_tiles) return;
    const TileDev t = p.tiles[tile];
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
    if (lane == 0) p.tcnt[tile] = (int32_t)n;
}

__global__ __launch_bounds__(256) void filt_write(FilterParams p) {
    const int lane = threadIdx.x & 63;
    const int tile = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (tile >= p.n_tiles) return;
    const TileDev t = p.tiles[tile];
    const SegDev seg = p.segs[t.seg];
    const uint64_t* abits = p.accept[t.seg];
    // this tile's offset inside its segment's list = Σ counts of the segment's earlier tiles (≤ a few
    // hundred L2-resident ints: cheaper than a separate prefix launch); the segment's last tile
    // publishes the segment's total
    const int2 st = p.seg_tiles[t.seg];
    int64_t off = 0;
    const int n_before = tile - st.x;
    for (int b = 0; b < n_before; b += 64 * 8) {   // 8 independent loads in flight per lane
        int v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int u = b + j * 64 + lane;
            v[j] = u < n_before ? p.tcnt[st.x + u] : 0;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) off += v[j];
    }
    for (int o = 32; o >= 1; o >>= 1) off += __shfl_xor(off, o);
    if (lane == 0 && tile == st.y - 1) p.scnt[t.seg] = (int32_t)(off + p.tcnt[tile]);
    uint32_t* out = p.comp + p.seg_vrow[t.seg];
    if (abits && seg.ord_to_doc) {   // sparse field: accept by doc, one 64-row window per step
        for (int64_t w0 = t.row_begin; w0 < t.row_end; w0 += 64) {
            const uint64_t m = __ballot(w0 + lane < t.row_end && accepted(abits, seg.ord_to_doc, w0 + lane));
            if ((m >> lane) & 1ull) out[off + __popcll(m & ((1ull << lane) - 1ull))] = (uint32_t)(w0 + lane);
            off += __popcll(m);
        }
        return;
    }
    // dense field: lane w loads the mask of window w of this pass of 64 windows (one load round trip),
    // a wave scan of their popcounts gives every window's output position, then the windows are
    // written one after the other from registers (no load in the loop)
    for (int64_t pb = t.row_begin; pb < t.row_end; pb += 64 * 64) {
        const int64_t w0 = pb + (int64_t)lane * 64;
        uint64_t m = 0ull;
        if (w0 < t.row_end) {
            const int64_t left = t.row_end - w0;
            m = abits ? window_mask(abits, w0, t.row_end) : (left >= 64 ? ~0ull : (1ull << left) - 1ull);
        }
        const int c = __popcll(m);
        int incl = c;
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
        }
        const int excl = incl - c;
        const int nw = (int)min<int64_t>(64, (t.row_end - pb + 63) / 64);
        for (int w = 0; w < nw; ++w) {
            const uint64_t mw = readlane64(m, w);
            const int base = __builtin_amdgcn_readlane(excl, w);
            if ((mw >> lane) & 1ull)
                out[off + base + __popcll(mw & ((1ull << lane) - 1ull))] = (uint32_t)(pb + (int64_t)w * 64 + lane);
        }
        off += __builtin_amdgcn_readlane(incl, 63);
    }
}

}  // namespace

hipError_t launch_filter_compact(const FilterParams& p, hipStream_t s) {
    if (p.n_tiles <= 0) return hipSuccess;
    const unsigned grid = (unsigned)((p.n_tiles + 3) / 4);
    hipLaunchKernelGGL(filt_count, dim3(grid), dim3(256), 0, s, p);
    hipLaunchKernelGGL(filt_write, dim3(grid), dim3(256), 0, s, p);
    return hipGetLastError();
}

}  // namespace osk
