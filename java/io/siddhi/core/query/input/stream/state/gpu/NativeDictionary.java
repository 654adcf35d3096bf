/*
 * NativeDictionary — a string -> dense id dictionary held by libsiddhi_hip.so (shp_dict), with a
 * lock-free Java cache in front.  Two uses per GPU query runtime:
 *   * string values: the SiddhiQL lowering (shp_compile_siddhiql) interns the filters' string
 *     constants here, and ColumnarBatch encodes string attribute values with the same ids, so
 *     `symbol == 'IBM'` compares ids that agree;
 *   * partition keys: bounded by cfg.max_keys (shp_dict_create(max_keys)); a new key past that
 *     many fails loudly (SHP_ERR_KEYS) instead of handing the engine an id it has no state for.
 *     Replaces the per-key state map of PartitionStateHolder.getState
 *     (core/util/snapshot/state/PartitionStateHolder.java:43-48) for this query.
 * Ids are assigned by the library under its own lock, so two threads interning new strings at
 * once get distinct ids (the cache only memoises what the library returned).
 * Source only: no JDK in this repository's image (DESIGN.md §6).
 */
package io.siddhi.core.query.input.stream.state.gpu;

import io.siddhi.core.exception.SiddhiAppRuntimeException;

import java.lang.foreign.Arena;
import java.lang.foreign.MemorySegment;
import java.nio.charset.StandardCharsets;
import java.util.concurrent.ConcurrentHashMap;

import static java.lang.foreign.ValueLayout.JAVA_BYTE;

final class NativeDictionary implements AutoCloseable {

    private final MemorySegment dict;   // shp_dict*
    private final ConcurrentHashMap<String, Integer> cache = new ConcurrentHashMap<>();
    private final String what;

    /** maxIds > 0: at most that many distinct strings (a partition-key dictionary: cfg.max_keys). */
    NativeDictionary(int maxIds, String what) {
        this.what = what;
        try {
            dict = (MemorySegment) ShpNative.DICT_CREATE.invokeExact(maxIds);
        } catch (Throwable t) {
            throw new IllegalStateException("shp_dict_create failed: " + t, t);
        }
    }

    MemorySegment handle() {
        return dict;
    }

    int id(String s) {
        Integer v = cache.get(s);
        if (v != null) {
            return v;
        }
        int id;
        try (Arena a = Arena.ofConfined()) {
            byte[] b = s.getBytes(StandardCharsets.UTF_8);
            MemorySegment seg = a.allocateFrom(JAVA_BYTE, b);
            id = (int) ShpNative.DICT_INTERN.invokeExact(dict, seg, (long) b.length);
        } catch (Throwable t) {
            throw new SiddhiAppRuntimeException("shp_dict_intern failed: " + t, t);
        }
        if (id < 0) {
            throw new SiddhiAppRuntimeException(what + ": " + ShpNative.codeName(id)
                    + " (more distinct values than the engine was created for)");
        }
        cache.putIfAbsent(s, id);
        return id;
    }

    @Override
    public void close() {
        try {
            ShpNative.DICT_DESTROY.invokeExact(dict);
        } catch (Throwable t) {
            throw new IllegalStateException("shp_dict_destroy failed: " + t, t);
        }
    }
}
