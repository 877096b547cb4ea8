/*
 * Panama FFM downcalls into libosknn.so (include/osknn.h).  Every entry point returns < 0 on failure and
 * osk_last_error() holds the message: check() turns it into an IOException, which OpenSearch reports as a
 * shard failure (S/search/query/QueryPhase.java:307-309).  The library never aborts.
 */
package org.opensearch.knn.gpu;

import java.io.IOException;
import java.lang.foreign.Arena;
import java.lang.foreign.FunctionDescriptor;
import java.lang.foreign.Linker;
import java.lang.foreign.MemorySegment;
import java.lang.foreign.SymbolLookup;
import java.lang.invoke.MethodHandle;

import static java.lang.foreign.ValueLayout.ADDRESS;
import static java.lang.foreign.ValueLayout.JAVA_FLOAT;
import static java.lang.foreign.ValueLayout.JAVA_INT;
import static java.lang.foreign.ValueLayout.JAVA_LONG;

final class OsKnn {
    private OsKnn() {}

    static final int OSK_FLOAT32 = 0;
    static final int OSK_BYTE = 1;
    static final int OSK_WARM_PREFILTER_MFMA = 2;
    static final int OSK_COMM_ID_BYTES = 128;

    private static final Linker LINKER = Linker.nativeLinker();
    private static final SymbolLookup LIB = SymbolLookup.libraryLookup(
        System.getProperty("osknn.library", "libosknn.so"), Arena.global());

    static MethodHandle h(String name, FunctionDescriptor fd, Linker.Option... options) {
        return LINKER.downcallHandle(LIB.find(name).orElseThrow(() -> new UnsatisfiedLinkError(name)), fd, options);
    }

    // const char* osk_last_error(void)
    static final MethodHandle LAST_ERROR = h("osk_last_error", FunctionDescriptor.of(ADDRESS));
    // int32_t osk_abi_version(void)
    static final MethodHandle ABI_VERSION = h("osk_abi_version", FunctionDescriptor.of(JAVA_INT));
    // int32_t osk_tune_set(const char* key, int64_t value)
    static final MethodHandle TUNE_SET = h("osk_tune_set", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_LONG));

    // int32_t osk_seg_stage(int32_t device, const void* rows, int64_t n_rows, int32_t dim, int32_t encoding,
    //                       int32_t similarity, const int32_t* ord_to_doc, int32_t max_doc, osk_seg** out)
    static final MethodHandle SEG_STAGE = h("osk_seg_stage", FunctionDescriptor.of(JAVA_INT,
        JAVA_INT, ADDRESS, JAVA_LONG, JAVA_INT, JAVA_INT, JAVA_INT, ADDRESS, JAVA_INT, ADDRESS));
    // int32_t osk_seg_stage_file(int32_t device, const char* path, int64_t data_offset, int64_t n_rows,
    //                            int32_t dim, int32_t encoding, int32_t similarity, const int32_t* ord_to_doc,
    //                            int32_t max_doc, osk_seg** out)
    static final MethodHandle SEG_STAGE_FILE = h("osk_seg_stage_file", FunctionDescriptor.of(JAVA_INT,
        JAVA_INT, ADDRESS, JAVA_LONG, JAVA_LONG, JAVA_INT, JAVA_INT, JAVA_INT, ADDRESS, JAVA_INT, ADDRESS));
    // int32_t osk_seg_search(osk_seg* seg, const void* queries, int32_t n_queries, int32_t k,
    //                        const uint64_t* accept_bits, float* out_scores, int32_t* out_docs,
    //                        int32_t* out_count, int64_t* out_visited)
    static final MethodHandle SEG_SEARCH = h("osk_seg_search", FunctionDescriptor.of(JAVA_INT,
        ADDRESS, ADDRESS, JAVA_INT, JAVA_INT, ADDRESS, ADDRESS, ADDRESS, ADDRESS, ADDRESS),
        Linker.Option.critical(true));   // heap arrays are passed directly
    static final MethodHandle SEG_RETAIN = h("osk_seg_retain", FunctionDescriptor.of(JAVA_INT, ADDRESS));
    static final MethodHandle SEG_RELEASE = h("osk_seg_release", FunctionDescriptor.of(JAVA_INT, ADDRESS));
    // int32_t osk_seg_footprint(const osk_seg* seg, int64_t* hbm_bytes)
    static final MethodHandle SEG_FOOTPRINT = h("osk_seg_footprint", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS));
    // int32_t osk_seg_warm(osk_seg* seg, int32_t what)
    static final MethodHandle SEG_WARM = h("osk_seg_warm", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT));

    // int32_t osk_view_create(osk_seg* const* segs, int32_t n_segs, const int32_t* seg_shard,
    //                         const int32_t* seg_doc_base, int32_t n_shards, const int32_t* shard_index,
    //                         osk_view** out)
    static final MethodHandle VIEW_CREATE = h("osk_view_create", FunctionDescriptor.of(JAVA_INT,
        ADDRESS, JAVA_INT, ADDRESS, ADDRESS, JAVA_INT, ADDRESS, ADDRESS));
    static final MethodHandle VIEW_RELEASE = h("osk_view_release", FunctionDescriptor.of(JAVA_INT, ADDRESS));
    // int32_t osk_view_search(osk_view* view, const void* queries, int32_t n_queries, int32_t k, int32_t from,
    //     int32_t size, const uint64_t* const* accept, float* out_scores, int32_t* out_docs,
    //     int32_t* out_shard_index, int32_t* out_count, int64_t* out_total_hits, float* out_max_score)
    static final MethodHandle VIEW_SEARCH = h("osk_view_search", FunctionDescriptor.of(JAVA_INT,
        ADDRESS, ADDRESS, JAVA_INT, JAVA_INT, JAVA_INT, JAVA_INT, ADDRESS, ADDRESS, ADDRESS, ADDRESS,
        ADDRESS, ADDRESS, ADDRESS));
    // int32_t osk_last_call_device_ns(int64_t* device_ns, int32_t* shared_by)
    static final MethodHandle LAST_CALL_NS = h("osk_last_call_device_ns", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS));

    // multi-GPU node (INTEGRATION.md §4)
    static final MethodHandle COMM_UNIQUE_ID = h("osk_comm_unique_id", FunctionDescriptor.of(JAVA_INT, ADDRESS));
    static final MethodHandle COMM_INIT_RANK = h("osk_comm_init_rank", FunctionDescriptor.of(JAVA_INT,
        JAVA_INT, JAVA_INT, JAVA_INT, ADDRESS, ADDRESS));
    static final MethodHandle COMM_INIT_ALL = h("osk_comm_init_all", FunctionDescriptor.of(JAVA_INT,
        ADDRESS, JAVA_INT, ADDRESS));
    static final MethodHandle COMM_RELEASE = h("osk_comm_release", FunctionDescriptor.of(JAVA_INT, ADDRESS));
    static final MethodHandle COMM_SET_DEVICE_LIMITS = h("osk_comm_set_device_limits", FunctionDescriptor.of(JAVA_INT,
        ADDRESS, JAVA_INT, JAVA_INT, JAVA_INT));
    static final MethodHandle SHARDS_SEARCH_MERGE = h("osk_shards_search_merge", FunctionDescriptor.of(JAVA_INT,
        ADDRESS, ADDRESS, JAVA_INT, ADDRESS, JAVA_INT, JAVA_INT, ADDRESS, JAVA_INT, JAVA_INT,
        ADDRESS, ADDRESS, ADDRESS, ADDRESS, ADDRESS, ADDRESS), Linker.Option.critical(true));

    // Lucene.writeTopDocs / readTopDocs, type 0 (S/common/lucene/Lucene.java:314-357, 407-447)
    static final MethodHandle TOPDOCS_WRITE = h("osk_topdocs_write", FunctionDescriptor.of(JAVA_INT,
        JAVA_LONG, JAVA_INT, JAVA_FLOAT, JAVA_INT, ADDRESS, ADDRESS, ADDRESS, JAVA_LONG, ADDRESS),
        Linker.Option.critical(true));

    static void check(int rc) throws IOException {
        if (rc != 0) {
            MemorySegment msg;
            try {
                msg = ((MemorySegment) LAST_ERROR.invokeExact()).reinterpret(4096);
            } catch (Throwable t) {
                throw new IOException("libosknn error " + rc, t);
            }
            throw new IOException("libosknn error " + rc + ": " + msg.getString(0));
        }
    }

    static IOException wrap(Throwable t) {
        if (t instanceof IOException io) return io;
        if (t instanceof RuntimeException re) throw re;
        if (t instanceof Error e) throw e;
        return new IOException(t);
    }

    /** This thread's last host search's device time in ns; −1 when the "call_timing" knob is off. */
    static long lastCallDeviceNs() {
        try (Arena a = Arena.ofConfined()) {
            MemorySegment ns = a.allocate(JAVA_LONG);
            check((int) LAST_CALL_NS.invokeExact(ns, MemorySegment.NULL));
            return ns.get(JAVA_LONG, 0);
        } catch (Throwable t) {
            return -1;
        }
    }

    static void tune(String key, long value) throws IOException {
        try (Arena a = Arena.ofConfined()) {
            check((int) TUNE_SET.invokeExact(a.allocateFrom(key), value));
        } catch (Throwable t) {
            throw wrap(t);
        }
    }
}
