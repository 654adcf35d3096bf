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
    private final ConcurrentHashMap<Integer, String> names = new ConcurrentHashMap<>();
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
        names.putIfAbsent(id, s);
        return id;
    }

    /** The string of id `id` (a match's partition key: the flow it is delivered in).  Ids this
     * process interned are cached; any other comes from the library (shp_dict_string). */
    String string(int id) {
        String s = names.get(id);
        if (s != null) {
            return s;
        }
        try (Arena a = Arena.ofConfined()) {
            long len = (long) ShpNative.DICT_STRING.invokeExact(dict, id, MemorySegment.NULL, 0L);
            if (len < 0) {
                throw new SiddhiAppRuntimeException(what + ": no string for id " + id + " ("
                        + ShpNative.codeName((int) len) + ")");
            }
            MemorySegment out = a.allocate(len + 1);
            long got = (long) ShpNative.DICT_STRING.invokeExact(dict, id, out, len + 1);
            s = new String(out.asSlice(0, len).toArray(JAVA_BYTE), StandardCharsets.UTF_8);
        } catch (RuntimeException e) {
            throw e;
        } catch (Throwable t) {
            throw new SiddhiAppRuntimeException("shp_dict_string failed: " + t, t);
        }
        names.putIfAbsent(id, s);
        return s;
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
