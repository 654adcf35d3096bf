/*
 * The columnar converter (SURVEY.md §8f-2): replaces StreamEventConverter
 * (core/event/stream/converter/StreamEventConverter.java) on the state path.  Receivers append
 * each arriving event straight into off-heap SoA columns (MemorySegments of a shared Arena) in
 * the layout shp_batch describes — ts:int64, key:int32 (partition-key dictionary id), stream:int32
 * (index in the program's "streams"), one column per program column (int->int32, long->int64,
 * float->float32, double->float64, bool->uint8, string->int32 dictionary id) with a null byte per
 * event — and keeps the rows so StateEvents can be rebuilt from the sequence numbers the engine
 * returns (StreamEvents are rebuilt from the batch rows, never copied back from the device).
 * Source only: no JDK in this repository's image (DESIGN.md §6).
 */
package io.siddhi.core.query.input.stream.state.gpu;

import io.siddhi.core.event.stream.StreamEvent;

import java.lang.foreign.Arena;
import java.lang.foreign.MemorySegment;
import java.lang.foreign.ValueLayout;
import java.util.ArrayDeque;
import java.util.ArrayList;
import java.util.List;

import static java.lang.foreign.ValueLayout.ADDRESS;
import static java.lang.foreign.ValueLayout.JAVA_BYTE;
import static java.lang.foreign.ValueLayout.JAVA_DOUBLE;
import static java.lang.foreign.ValueLayout.JAVA_FLOAT;
import static java.lang.foreign.ValueLayout.JAVA_INT;
import static java.lang.foreign.ValueLayout.JAVA_LONG;

final class ColumnarBatch {

    /** program["columns"][c]: (stream index, attribute position in that stream, type tag). */
    static final class Column {
        final int stream;
        final int attr;
        final char type;  // 'i' int, 'l' long, 'f' float, 'd' double, 'b' bool, 's' string id

        Column(int stream, int attr, char type) {
            this.stream = stream;
            this.attr = attr;
            this.type = type;
        }

        int bytes() {
            return type == 'l' || type == 'd' ? 8 : (type == 'b' ? 1 : 4);
        }
    }

    private final Arena arena;
    private final long capacity;
    private final Column[] columns;
    private final MemorySegment ts, key, stream;
    private final MemorySegment[] cols, nulls;
    private final MemorySegment colPtrs, nullPtrs, descriptor;
    private final NativeDictionary strings;           // string-attribute dictionary (shared with the filters)
    private long n;
    private long seq0;                                // sequence number of row 0 of this batch
    // rows of earlier batches still referenced by open partial matches: the engine reports match
    // slots as sequence numbers, which may point into any earlier push (every e1 waiting for e2)
    private final ArrayDeque<Object[][]> history = new ArrayDeque<>();
    private final ArrayDeque<long[]> historySeq = new ArrayDeque<>();
    private final int historyBatches;
    private final List<Object[]> rows = new ArrayList<>();
    private final List<long[]> rowMeta = new ArrayList<>();  // {ts, stream}

    ColumnarBatch(Arena arena, long capacity, Column[] columns, NativeDictionary strings, int historyBatches) {
        this.arena = arena;
        this.capacity = capacity;
        this.columns = columns;
        this.strings = strings;
        this.historyBatches = historyBatches;
        ts = arena.allocate(JAVA_LONG, capacity);
        key = arena.allocate(JAVA_INT, capacity);
        stream = arena.allocate(JAVA_INT, capacity);
        cols = new MemorySegment[columns.length];
        nulls = new MemorySegment[columns.length];
        colPtrs = arena.allocate(ADDRESS, Math.max(1, columns.length));
        nullPtrs = arena.allocate(ADDRESS, Math.max(1, columns.length));
        for (int c = 0; c < columns.length; c++) {
            cols[c] = arena.allocate(columns[c].bytes() * capacity, 8);
            nulls[c] = arena.allocate(JAVA_BYTE, capacity);
            colPtrs.setAtIndex(ADDRESS, c, cols[c]);
            nullPtrs.setAtIndex(ADDRESS, c, nulls[c]);
        }
        descriptor = arena.allocate(ShpNative.BATCH);
    }

    boolean full() {
        return n >= capacity;
    }

    long size() {
        return n;
    }

    /** Appends one event (InputHandler.send -> Receiver.receive).  keyId: the partition-key
     * dictionary id (PartitionStreamReceiver's key string, ValuePartitionExecutor.execute), 0 when
     * the query is not partitioned; streamIndex: -1 for a clock-only event (a send on a stream this
     * query does not read, which in playback still sets the app's clock). */
    void append(long timestamp, int keyId, int streamIndex, Object[] data) {
        ts.setAtIndex(JAVA_LONG, n, timestamp);
        key.setAtIndex(JAVA_INT, n, keyId);
        stream.setAtIndex(JAVA_INT, n, streamIndex);
        for (int c = 0; c < columns.length; c++) {
            Column col = columns[c];
            Object v = (streamIndex == col.stream && data != null) ? data[col.attr] : null;
            nulls[c].set(JAVA_BYTE, n, (byte) (v == null ? 1 : 0));
            if (v == null) {
                continue;
            }
            switch (col.type) {
                case 'i': cols[c].setAtIndex(JAVA_INT, n, ((Number) v).intValue()); break;
                case 'l': cols[c].setAtIndex(JAVA_LONG, n, ((Number) v).longValue()); break;
                case 'f': cols[c].setAtIndex(JAVA_FLOAT, n, ((Number) v).floatValue()); break;
                case 'd': cols[c].setAtIndex(JAVA_DOUBLE, n, ((Number) v).doubleValue()); break;
                case 'b': cols[c].set(JAVA_BYTE, n, (byte) (((Boolean) v) ? 1 : 0)); break;
                default: cols[c].setAtIndex(JAVA_INT, n, strings.id(v.toString())); break;
            }
        }
        rows.add(data);
        rowMeta.add(new long[]{timestamp, streamIndex});
        n++;
    }

    /** The shp_batch descriptor of the rows appended so far (host memory; shp_push_batch copies it). */
    MemorySegment descriptor() {
        descriptor.set(JAVA_LONG, 0, n);
        descriptor.set(ADDRESS, 8, ts);
        descriptor.set(ADDRESS, 16, key);
        descriptor.set(ADDRESS, 24, stream);
        descriptor.set(ADDRESS, 32, colPtrs);
        descriptor.set(ADDRESS, 40, nullPtrs);
        descriptor.set(ADDRESS, 48, MemorySegment.NULL);  // clock: the events' own ts
        descriptor.set(ADDRESS, 56, MemorySegment.NULL);  // seq: the engine's running count
        return descriptor;
    }

    /** After a failed push: the engine did not take the rows (its sequence counter did not move),
     * so they are dropped and row 0 of the next batch keeps this batch's seq0. */
    void discard() {
        n = 0;
        rows.clear();
        rowMeta.clear();
    }

    /** After a successful push: the rows move to the history (matches of later pushes may name them). */
    void clear() {
        history.addLast(rows.toArray(new Object[0][]));
        long[] meta = new long[rows.size() * 2 + 1];
        meta[0] = seq0;
        for (int i = 0; i < rowMeta.size(); i++) {
            meta[1 + 2 * i] = rowMeta.get(i)[0];
            meta[2 + 2 * i] = rowMeta.get(i)[1];
        }
        historySeq.addLast(meta);
        while (history.size() > historyBatches) {
            history.removeFirst();
            historySeq.removeFirst();
        }
        seq0 += n;
        n = 0;
        rows.clear();
        rowMeta.clear();
    }

    /** The StreamEvent of sequence number `seq` (a match slot), rebuilt from the kept row, with the
     * before-window data the query's MetaStreamEvent expects for that stream. */
    StreamEvent event(long seq, int outputDataSize) {
        Object[][] block = null;
        long[] meta = null;
        var hit = history.descendingIterator();
        var hitSeq = historySeq.descendingIterator();
        while (hit.hasNext()) {
            Object[][] b = hit.next();
            long[] m = hitSeq.next();
            if (seq >= m[0] && seq < m[0] + b.length) {
                block = b;
                meta = m;
                break;
            }
        }
        if (block == null) {
            throw new IllegalStateException("event " + seq + " is older than the kept history (" + historyBatches
                    + " pushes); raise the history or add `within` to the query");
        }
        int i = (int) (seq - meta[0]);
        Object[] data = block[i];
        StreamEvent e = new StreamEvent(0, 0, outputDataSize);
        e.setTimestamp(meta[1 + 2 * i]);
        e.setOutputData(data.clone());
        return e;
    }

    long nextSeq() {
        return seq0 + n;
    }

    @SuppressWarnings("unused")
    private static final ValueLayout.OfLong LONG = JAVA_LONG;
}
