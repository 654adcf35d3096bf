/*
 * Panama FFM (java.lang.foreign, JDK >= 22) binding of libsiddhi_hip.so — include/siddhi_hip.h.
 * Source only: this repository's image has no JDK, so it is not compiled here (DESIGN.md §6).
 *
 * Every downcall mirrors one C-ABI entry point; struct layouts mirror shp_config, shp_batch and
 * shp_matches field for field.  tests/test_java_binding.py parses the layouts and the CFG_* offsets
 * below out of this file and checks them against the header compiled with gcc (offsetof), and
 * checks that every symbol a downcall names is declared in include/siddhi_hip.h.
 */
package io.siddhi.core.query.input.stream.state.gpu;

import java.lang.foreign.Arena;
import java.lang.foreign.FunctionDescriptor;
import java.lang.foreign.Linker;
import java.lang.foreign.MemoryLayout;
import java.lang.foreign.MemorySegment;
import java.lang.foreign.StructLayout;
import java.lang.foreign.SymbolLookup;
import java.lang.invoke.MethodHandle;

import static java.lang.foreign.ValueLayout.ADDRESS;
import static java.lang.foreign.ValueLayout.JAVA_DOUBLE;
import static java.lang.foreign.ValueLayout.JAVA_INT;
import static java.lang.foreign.ValueLayout.JAVA_LONG;

final class ShpNative {

    static final int OK = 0;
    static final int ERR_ARG = -1;
    static final int ERR_UNSUPPORTED = -2;
    static final int ERR_CAPACITY = -3;
    static final int ERR_OUTPUT = -4;
    static final int ERR_DEVICE = -5;
    static final int ERR_KEYS = -6;

    static final int LAYOUT_FULL = 0;
    static final int LAYOUT_PAIRS = 1;
    static final int LAYOUT_AGG = 2;
    static final int LAYOUT_PAIRS32 = 3;
    /** count-sequence path: one uint32 per match, e2's batch index | L << 28 (include/siddhi_hip.h). */
    static final int LAYOUT_CHAIN32 = 4;
    /** the engine's own compact form, resolved at create (PAIRS32 / CHAIN32 / FULL; shp_engine_stat "match_layout"). */
    static final int LAYOUT_COMPACT = 5;

    static final int COMM_ID_BYTES = 128;

    static final Linker LINKER = Linker.nativeLinker();
    static final SymbolLookup LIB = SymbolLookup.libraryLookup(
            System.getProperty("siddhi.hip.lib", "libsiddhi_hip.so"), Arena.global());

    /** struct shp_config (48 bytes). */
    static final StructLayout CONFIG = MemoryLayout.structLayout(
            JAVA_INT.withName("device"), JAVA_INT.withName("max_keys"),
            JAVA_LONG.withName("max_batch"), JAVA_LONG.withName("max_matches"),
            JAVA_LONG.withName("start_clock"), JAVA_INT.withName("force_general"),
            JAVA_INT.withName("profile_kernels"), JAVA_INT.withName("match_layout"),
            MemoryLayout.paddingLayout(4));

    /** Field offsets of shp_config (GpuStateStreamRuntime fills the struct by offset). */
    static final long CFG_DEVICE = 0, CFG_MAX_KEYS = 4, CFG_MAX_BATCH = 8, CFG_MAX_MATCHES = 16,
            CFG_START_CLOCK = 24, CFG_FORCE_GENERAL = 32, CFG_PROFILE_KERNELS = 36, CFG_MATCH_LAYOUT = 40;

    /** struct shp_batch (64 bytes): n, ts, key, stream, cols, nulls, clock, seq. */
    static final StructLayout BATCH = MemoryLayout.structLayout(
            JAVA_LONG.withName("n"), ADDRESS.withName("ts"), ADDRESS.withName("key"),
            ADDRESS.withName("stream"), ADDRESS.withName("cols"), ADDRESS.withName("nulls"),
            ADDRESS.withName("clock"), ADDRESS.withName("seq"));

    /** struct shp_matches (88 bytes). */
    static final StructLayout MATCHES = MemoryLayout.structLayout(
            JAVA_LONG.withName("m"), JAVA_INT.withName("num_states"), MemoryLayout.paddingLayout(4),
            ADDRESS.withName("key"), ADDRESS.withName("ts"), ADDRESS.withName("type"),
            ADDRESS.withName("pos"), ADDRESS.withName("ref_off"), ADDRESS.withName("slot_len"),
            ADDRESS.withName("refs"), JAVA_INT.withName("layout"), MemoryLayout.paddingLayout(4),
            ADDRESS.withName("agg"));

    // ---- one engine (StateInputStreamParser.parseInputStream + the processor chain)
    static final MethodHandle ENGINE_CREATE = fn("shp_engine_create", JAVA_INT, ADDRESS, ADDRESS, ADDRESS);
    static final MethodHandle PUSH_BATCH = fn("shp_push_batch", JAVA_INT, ADDRESS, ADDRESS, ADDRESS);
    static final MethodHandle PUSH_BATCH_DEVICE = fn("shp_push_batch_device", JAVA_INT, ADDRESS, ADDRESS, ADDRESS);
    // host push, records in the engine's compact layout (no expansion): the runtime's push
    static final MethodHandle PUSH_BATCH_COMPACT = fn("shp_push_batch_compact", JAVA_INT, ADDRESS, ADDRESS, ADDRESS);
    // the oldest event an open partial still holds: the rows below it may be dropped (ColumnarBatch.trim)
    static final MethodHandle OLDEST_LIVE_SEQ = fn("shp_engine_oldest_live_seq", JAVA_INT, ADDRESS, ADDRESS);
    // pipelined host ingest: H2D of the next batch on the engine's copy stream while it runs the staged one
    static final MethodHandle STAGE_BATCH = fn("shp_stage_batch", JAVA_INT, ADDRESS, ADDRESS);
    static final MethodHandle STAGE_BATCH_TS32 = fn("shp_stage_batch_ts32", JAVA_INT, ADDRESS, ADDRESS, JAVA_LONG,
            ADDRESS);
    static final MethodHandle STAGE_BATCH_NARROW = fn("shp_stage_batch_narrow", JAVA_INT, ADDRESS, ADDRESS, JAVA_LONG,
            ADDRESS, ADDRESS);
    static final MethodHandle RUN_STAGED = fn("shp_run_staged", JAVA_INT, ADDRESS, ADDRESS);
    // the earliest head of any key's timer queue: a live-mode runtime's wall-clock wake-up (Scheduler.schedule)
    static final MethodHandle NEXT_DUE = fn("shp_engine_next_due", JAVA_INT, ADDRESS, ADDRESS);
    static final MethodHandle FETCH_MATCHES = fn("shp_fetch_matches", JAVA_INT, ADDRESS, ADDRESS);
    static final MethodHandle ADVANCE_CLOCK = fn("shp_advance_clock", JAVA_INT, ADDRESS, JAVA_LONG, ADDRESS);
    static final MethodHandle SNAPSHOT = fn("shp_snapshot", JAVA_INT, ADDRESS, ADDRESS, ADDRESS);
    static final MethodHandle RESTORE = fn("shp_restore", JAVA_INT, ADDRESS, ADDRESS, JAVA_LONG);
    static final MethodHandle SNAPSHOT_DESCRIBE = fn("shp_snapshot_describe", JAVA_LONG, ADDRESS, ADDRESS, JAVA_LONG,
            ADDRESS, JAVA_LONG);
    static final MethodHandle NUM_STATES = fn("shp_engine_num_states", JAVA_INT, ADDRESS);
    // the stream (program order) a state reads: one SingleStreamRuntime per state on that receiver
    static final MethodHandle STATE_STREAM = fn("shp_engine_state_stream", JAVA_INT, ADDRESS, JAVA_INT);
    static final MethodHandle ENGINE_PATH = fn("shp_engine_path", JAVA_INT, ADDRESS);
    static final MethodHandle ENGINE_STAT = fn("shp_engine_stat", JAVA_LONG, ADDRESS, ADDRESS);  // monitoring counters
    static final MethodHandle LAST_ERROR = fn("shp_last_error", ADDRESS, ADDRESS);
    static final MethodHandle ENGINE_DESTROY = fnVoid("shp_engine_destroy", ADDRESS);

    // ---- SiddhiQL lowering inside the library (StateInputStreamParser.parse + ExpressionParser)
    static final MethodHandle DICT_CREATE = fn("shp_dict_create", ADDRESS, JAVA_INT);
    static final MethodHandle DICT_INTERN = fn("shp_dict_intern", JAVA_INT, ADDRESS, ADDRESS, JAVA_LONG);
    static final MethodHandle DICT_SIZE = fn("shp_dict_size", JAVA_INT, ADDRESS);
    static final MethodHandle DICT_STRING = fn("shp_dict_string", JAVA_LONG, ADDRESS, JAVA_INT, ADDRESS, JAVA_LONG);
    static final MethodHandle DICT_DESTROY = fnVoid("shp_dict_destroy", ADDRESS);
    static final MethodHandle COMPILE_SIDDHIQL = fn("shp_compile_siddhiql", JAVA_LONG, ADDRESS, ADDRESS, ADDRESS,
            ADDRESS, JAVA_LONG);
    static final MethodHandle SIDDHIQL_QUERIES = fn("shp_siddhiql_queries", JAVA_LONG, ADDRESS, ADDRESS, JAVA_LONG);
    static final MethodHandle COMPILE_LAST_ERROR = fn("shp_compile_last_error", ADDRESS);
    static final MethodHandle ENGINE_CREATE_SIDDHIQL = fn("shp_engine_create_siddhiql", JAVA_INT, ADDRESS, ADDRESS,
            ADDRESS, ADDRESS, ADDRESS);

    // ---- page-locked receive memory for match payloads
    static final MethodHandle HOST_REGISTER = fn("shp_host_register", JAVA_INT, ADDRESS, JAVA_LONG);
    static final MethodHandle HOST_UNREGISTER = fn("shp_host_unregister", JAVA_INT, ADDRESS);

    // ---- key-sharded groups (multi-GPU behind the C-ABI)
    static final MethodHandle COMM_ID = fn("shp_comm_id", JAVA_INT, ADDRESS, JAVA_LONG);
    static final MethodHandle GROUP_CREATE = fn("shp_group_create", JAVA_INT, ADDRESS, ADDRESS, JAVA_INT, ADDRESS,
            ADDRESS);
    static final MethodHandle GROUP_CREATE_RANK = fn("shp_group_create_rank", JAVA_INT, ADDRESS, ADDRESS, JAVA_INT,
            JAVA_INT, ADDRESS, ADDRESS);
    static final MethodHandle GROUP_PUSH = fn("shp_group_push", JAVA_INT, ADDRESS, ADDRESS, ADDRESS);
    static final MethodHandle GROUP_STAGE = fn("shp_group_stage", JAVA_INT, ADDRESS, ADDRESS);
    static final MethodHandle GROUP_RUN = fn("shp_group_run", JAVA_INT, ADDRESS, ADDRESS);
    static final MethodHandle GROUP_FETCH = fn("shp_group_fetch_matches", JAVA_INT, ADDRESS, ADDRESS);
    // collective: every rank's matches of the last push to rank `root` (int32), moved in HBM
    static final MethodHandle GROUP_GATHER = fn("shp_group_gather_matches", JAVA_INT, ADDRESS, JAVA_INT, ADDRESS);
    static final MethodHandle GROUP_LAST_ERROR = fn("shp_group_last_error", ADDRESS, ADDRESS);
    static final MethodHandle GROUP_DESTROY = fnVoid("shp_group_destroy", ADDRESS);

    private ShpNative() {
    }

    private static MethodHandle fn(String name, MemoryLayout ret, MemoryLayout... args) {
        return LINKER.downcallHandle(LIB.find(name).orElseThrow(
                () -> new UnsatisfiedLinkError("libsiddhi_hip.so does not export " + name)),
                FunctionDescriptor.of(ret, args));
    }

    private static MethodHandle fnVoid(String name, MemoryLayout... args) {
        return LINKER.downcallHandle(LIB.find(name).orElseThrow(
                () -> new UnsatisfiedLinkError("libsiddhi_hip.so does not export " + name)),
                FunctionDescriptor.ofVoid(args));
    }

    /** The engine's last error text (shp_last_error). */
    static String lastError(MemorySegment engine) {
        try {
            MemorySegment s = (MemorySegment) LAST_ERROR.invokeExact(engine);
            return s.reinterpret(1 << 16).getString(0);
        } catch (Throwable t) {
            return "shp_last_error failed: " + t;
        }
    }

    /** The calling thread's last lowering error (shp_compile_last_error). */
    static String compileLastError() {
        try {
            MemorySegment s = (MemorySegment) COMPILE_LAST_ERROR.invokeExact();
            return s.reinterpret(1 << 16).getString(0);
        } catch (Throwable t) {
            return "shp_compile_last_error failed: " + t;
        }
    }

    /** The program JSON of one query of a SiddhiQL app, lowered by the library (shp_compile_siddhiql);
     * string constants are interned in `dict`. */
    static String compileSiddhiQL(String appText, String queryName, NativeDictionary dict) {
        try (Arena a = Arena.ofConfined()) {
            MemorySegment app = a.allocateFrom(appText);
            MemorySegment q = queryName == null ? MemorySegment.NULL : a.allocateFrom(queryName);
            long n = (long) COMPILE_SIDDHIQL.invokeExact(app, q, dict.handle(), MemorySegment.NULL, 0L);
            if (n < 0) {
                throw new IllegalArgumentException(codeName((int) n) + ": " + compileLastError());
            }
            MemorySegment out = a.allocate(n + 1);
            long got = (long) COMPILE_SIDDHIQL.invokeExact(app, q, dict.handle(), out, n + 1);
            return out.getString(0);
        } catch (RuntimeException e) {
            throw e;
        } catch (Throwable t) {
            throw new IllegalStateException("shp_compile_siddhiql failed: " + t, t);
        }
    }

    static String groupLastError(MemorySegment group) {
        try {
            MemorySegment s = (MemorySegment) GROUP_LAST_ERROR.invokeExact(group);
            return s.reinterpret(1 << 16).getString(0);
        } catch (Throwable t) {
            return "shp_group_last_error failed: " + t;
        }
    }

    static String codeName(int rc) {
        switch (rc) {
            case ERR_ARG: return "SHP_ERR_ARG";
            case ERR_UNSUPPORTED: return "SHP_ERR_UNSUPPORTED";
            case ERR_CAPACITY: return "SHP_ERR_CAPACITY";
            case ERR_OUTPUT: return "SHP_ERR_OUTPUT";
            case ERR_DEVICE: return "SHP_ERR_DEVICE";
            case ERR_KEYS: return "SHP_ERR_KEYS";
            default: return Integer.toString(rc);
        }
    }

    /** Reads field `name` of an shp_matches the library filled. */
    static long matchesLong(MemorySegment m, String name) {
        return m.get(JAVA_LONG, MATCHES.byteOffset(MemoryLayout.PathElement.groupElement(name)));
    }

    static int matchesInt(MemorySegment m, String name) {
        return m.get(JAVA_INT, MATCHES.byteOffset(MemoryLayout.PathElement.groupElement(name)));
    }

    static MemorySegment matchesPtr(MemorySegment m, String name, long bytes) {
        return m.get(ADDRESS, MATCHES.byteOffset(MemoryLayout.PathElement.groupElement(name))).reinterpret(bytes);
    }

    static double aggAt(MemorySegment agg, long i) {
        return agg.getAtIndex(JAVA_DOUBLE, i);
    }
}
