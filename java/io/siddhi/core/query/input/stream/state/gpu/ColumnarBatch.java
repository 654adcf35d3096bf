/*
 * The columnar converter (SURVEY.md §8f-2): replaces StreamEventConverter
 * (core/event/stream/converter/StreamEventConverter.java) on the state path.  Receivers append
 * each arriving event straight into off-heap SoA columns (MemorySegments of a shared Arena) in
 * the layout shp_batch describes — ts:int64, key:int32 (partition-key dictionary id), stream:int32
 * (index in the program's "streams"), one column per program column (int->int32, long->int64,
 * float->float32, double->float64, bool->uint8, string->int32 dictionary id) with a null byte per
 * event — and keeps the rows so StateEvents can be rebuilt from the sequence numbers the engine
 * returns (StreamEvents are rebuilt from the batch rows, never copied back from the device).
 *
 * Retention: the reference keeps a StreamEvent alive exactly as long as a partial holds it
 * (StreamPreStateProcessor.java:364-403).  The rows of committed pushes are kept by sequence
 * number from shp_engine_oldest_live_seq on (the oldest event an open partial of the engine's
 * committed state holds): trim() drops everything below it, maybeTrim() asks the engine once the
 * kept rows have doubled since the last trim, so the query (a state snapshot) stays amortised.
 * The Python mirror of these rules is siddhi_amd/history.py (RowHistory), tested in
 * tests/test_retention.py.
 *
 * Pipelined ingest (FlushPolicy.PIPELINED): two column sets; a flush stages the filled set
 * (shp_stage_batch: its H2D copies on the engine's copy stream, from page-locked segments) and
 * runs the set staged before it (shp_run_staged), whose rows then join the history -- sequence
 * numbers follow run order, which is stage order.  The mirror is SiddhiAppRuntime(pipelined=True)
 * (siddhi_amd/runtime.py), tested in tests/test_flow_clock.py.  Source only: no JDK in this repository's image (DESIGN.md §6).
 */
package io.siddhi.core.query.input.stream.state.gpu;

import io.siddhi.core.event.stream.StreamEvent;

import java.lang.foreign.Arena;
import java.lang.foreign.MemorySegment;
import java.util.ArrayDeque;
import java.util.ArrayList;
import java.util.Arrays;
import java.util.List;
import java.util.function.LongSupplier;

import static java.lang.foreign.ValueLayout.ADDRESS;
import static java.lang.foreign.ValueLayout.JAVA_BYTE;
import static java.lang.foreign.ValueLayout.JAVA_DOUBLE;
import static java.lang.foreign.ValueLayout.JAVA_FLOAT;
import static java.lang.foreign.ValueLayout.JAVA_INT;
import static java.lang.foreign.ValueLayout.JAVA_LONG;
import static java.lang.foreign.ValueLayout.JAVA_SHORT;

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

    /** The rows of one committed push from sequence number seq0 on (a trimmed push keeps its tail). */
    static final class Block {
        final long seq0;
        final Object[][] rows;
        final long[] ts;

        Block(long seq0, Object[][] rows, long[] ts) {
            this.seq0 = seq0;
            this.rows = rows;
            this.ts = ts;
        }

        long end() {
            return seq0 + rows.length;
        }
    }

    /** One set of host columns in shp_batch's layout with the rows appended into it.  A DEFERRED /
     * SYNC batch has one; a PIPELINED batch two, so one set is being filled (or decoded) while the
     * other's H2D copies (shp_stage_batch, on the engine's copy stream) are in flight. */
    private final class Columns {
        final MemorySegment ts, key, stream;
        final MemorySegment[] cols, nulls;
        final MemorySegment colPtrs, nullPtrs, descriptor;
        final List<Object[]> rows = new ArrayList<>();
        final List<Long> rowTs = new ArrayList<>();
        long n;
        // the narrow form (shp_stage_batch_narrow): ts as 4-byte offsets from the batch's first ts and
        // 2-byte key ids, kept beside the wide columns; `wide` once an offset leaves the int range
        final MemorySegment ts32, key16;
        long base;
        boolean wide;

        Columns() {
            ts32 = narrow ? arena.allocate(JAVA_INT, capacity) : null;
            key16 = narrow ? arena.allocate(JAVA_SHORT, capacity) : null;
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

        List<MemorySegment> segments() {
            List<MemorySegment> l = new ArrayList<>(List.of(ts, key, stream));
            if (narrow) {
                l.add(ts32);
                l.add(key16);
            }
            l.addAll(Arrays.asList(cols));
            l.addAll(Arrays.asList(nulls));
            return l;
        }

        void clear() {
            n = 0;
            rows.clear();
            rowTs.clear();
        }
    }

    private final Arena arena;
    private final long capacity;
    private final Column[] columns;
    private final NativeDictionary strings;           // string-attribute dictionary (shared with the filters)
    private final boolean narrow;                     // PIPELINED with max_keys <= 65536: narrow columns too
    private Columns open;                             // the set appends go to (null only inside a flush)
    private Columns decoded;                          // the set of the last committed push (keyAt / tsAt / streamAt)
    private final ArrayDeque<Columns> staged = new ArrayDeque<>();  // PIPELINED: staged, oldest first
    private final ArrayDeque<Columns> free = new ArrayDeque<>();
    private final List<MemorySegment> pinned = new ArrayList<>();
    private long seq0;                                // sequence number of the oldest row not yet committed
    // rows of committed pushes still named by open partials (or not yet trimmed), oldest first:
    // blocks [head, size) of the list, ordered by seq0, so a match slot's row is found by bisection
    private final ArrayList<Block> history = new ArrayList<>();
    private int head;
    private long kept;                                // rows held in `history`
    private long floor;                               // every row below it was dropped
    private final long minTrim;
    private long trimAt;

    /** @param sets   1 (SYNC / DEFERRED) or 2 (PIPELINED: the second set fills while the first is staged)
     *  @param narrow keep the narrow form's columns too (key ids below 65536) */
    ColumnarBatch(Arena arena, long capacity, Column[] columns, NativeDictionary strings, long minTrim, int sets,
                  boolean narrow) {
        this.arena = arena;
        this.capacity = capacity;
        this.columns = columns;
        this.strings = strings;
        this.narrow = narrow;
        this.minTrim = Math.max(1, minTrim);
        this.trimAt = this.minTrim;
        open = new Columns();
        decoded = open;
        for (int i = 1; i < sets; i++) {
            free.add(new Columns());
        }
    }

    ColumnarBatch(Arena arena, long capacity, Column[] columns, NativeDictionary strings, long minTrim) {
        this(arena, capacity, columns, strings, minTrim, 1, false);
    }

    /** Page-locks every column segment (shp_host_register) so shp_stage_batch's copies run at DMA rate
     * and asynchronously; undone by unpin() before the arena closes. */
    void pin() throws Throwable {
        List<Columns> all = new ArrayList<>(free);
        all.add(open);
        for (Columns c : all) {
            for (MemorySegment m : c.segments()) {
                int rc = (int) ShpNative.HOST_REGISTER.invokeExact(m, m.byteSize());
                if (rc != ShpNative.OK) {
                    throw new IllegalStateException("shp_host_register: " + ShpNative.codeName(rc));
                }
                pinned.add(m);
            }
        }
    }

    void unpin() throws Throwable {
        for (MemorySegment m : pinned) {
            int rc = (int) ShpNative.HOST_UNREGISTER.invokeExact(m);   // best effort at close
        }
        pinned.clear();
    }

    boolean full() {
        return open.n >= capacity;
    }

    long size() {
        return open.n;
    }

    /** Appends one event (InputHandler.send -> Receiver.receive).  keyId: the partition-key
     * dictionary id (PartitionStreamReceiver's key string, ValuePartitionExecutor.execute), 0 when
     * the query is not partitioned; streamIndex: -1 for a clock-only event (a send on a stream this
     * query does not read, which in playback still sets the app's clock). */
    void append(long timestamp, int keyId, int streamIndex, Object[] data) {
        Columns o = open;
        long n = o.n;
        if (streamIndex >= 0 && n > 0 && o.stream.getAtIndex(JAVA_INT, n - 1) < 0
                && o.rowTs.get((int) n - 1) == timestamp) {
            // the clock-only row the query's TimeChangeListener appended for this very send
            // (InputHandler.send sets the clock before the event reaches the receiver): the event
            // carries the same clock, so it takes the row's place
            n--;
            o.rows.remove(o.rows.size() - 1);
            o.rowTs.remove(o.rowTs.size() - 1);
        }
        o.ts.setAtIndex(JAVA_LONG, n, timestamp);
        o.key.setAtIndex(JAVA_INT, n, keyId);
        if (narrow) {
            if (n == 0) {
                o.base = timestamp;
                o.wide = false;
            }
            long d = timestamp - o.base;
            if (d != (int) d) {
                o.wide = true;
            }
            o.ts32.setAtIndex(JAVA_INT, n, (int) d);
            o.key16.setAtIndex(JAVA_SHORT, n, (short) keyId);   // (ids < 65536: read back unsigned)
        }
        o.stream.setAtIndex(JAVA_INT, n, streamIndex);
        for (int c = 0; c < columns.length; c++) {
            Column col = columns[c];
            Object v = (streamIndex == col.stream && data != null) ? data[col.attr] : null;
            o.nulls[c].set(JAVA_BYTE, n, (byte) (v == null ? 1 : 0));
            if (v == null) {
                continue;
            }
            MemorySegment d = o.cols[c];
            switch (col.type) {
                case 'i': d.setAtIndex(JAVA_INT, n, ((Number) v).intValue()); break;
                case 'l': d.setAtIndex(JAVA_LONG, n, ((Number) v).longValue()); break;
                case 'f': d.setAtIndex(JAVA_FLOAT, n, ((Number) v).floatValue()); break;
                case 'd': d.setAtIndex(JAVA_DOUBLE, n, ((Number) v).doubleValue()); break;
                case 'b': d.set(JAVA_BYTE, n, (byte) (((Boolean) v) ? 1 : 0)); break;
                default: d.setAtIndex(JAVA_INT, n, strings.id(v.toString())); break;
            }
        }
        o.rows.add(data);
        o.rowTs.add(timestamp);
        o.n = n + 1;
    }

    /** A clock-only row (stream -1, no key, no values): the app clock moved to `now` with no event of
     * this query (a send on another stream, the playback heartbeat) -- GpuStateStreamRuntime's
     * TimeChangeListener under FlushPolicy.DEFERRED.  The engine fires the timers due by then. */
    void appendClock(long now) {
        append(now, 0, -1, null);
    }

    /** The shp_batch descriptor of the rows appended so far (host memory; shp_push_batch copies it,
     * shp_stage_batch reads it until the shp_run_staged that consumes it). */
    MemorySegment descriptor() {
        Columns o = open;
        o.descriptor.set(JAVA_LONG, 0, o.n);
        o.descriptor.set(ADDRESS, 8, o.ts);
        o.descriptor.set(ADDRESS, 16, o.key);
        o.descriptor.set(ADDRESS, 24, o.stream);
        o.descriptor.set(ADDRESS, 32, o.colPtrs);
        o.descriptor.set(ADDRESS, 40, o.nullPtrs);
        o.descriptor.set(ADDRESS, 48, MemorySegment.NULL);  // clock: the events' own ts
        o.descriptor.set(ADDRESS, 56, MemorySegment.NULL);  // seq: the engine's running count
        return o.descriptor;
    }

    /** The open rows can go in the narrow form (shp_stage_batch_narrow). */
    boolean narrowOk() {
        return narrow && open.n > 0 && !open.wide;
    }

    long narrowBase() {
        return open.base;
    }

    MemorySegment ts32() {
        return open.ts32;
    }

    MemorySegment key16() {
        return open.key16;
    }

    /** After a failed push or stage: the engine did not take the rows (its sequence counter did not
     * move), so they are dropped and row 0 of the next batch keeps this batch's seq0. */
    void discard() {
        open.clear();
    }

    /** After a successful push: the rows join the history (matches of this and later pushes name
     * them) and the batch is empty again.  The pushed key / ts / stream columns stay readable
     * (keyAt, tsAt, streamAt) until the next append: the compact records are decoded from them.
     * Returns the pushed rows' first sequence number. */
    long commit() {
        decoded = open;
        long first = commitRows(open);
        open.clear();
        return first;
    }

    private long commitRows(Columns c) {
        long first = seq0;
        if (c.n > 0) {
            long[] t = new long[c.rowTs.size()];
            for (int i = 0; i < t.length; i++) {
                t[i] = c.rowTs.get(i);
            }
            history.add(new Block(seq0, c.rows.toArray(new Object[0][]), t));
            kept += c.n;
        }
        seq0 += c.n;
        return first;
    }

    // ---- PIPELINED (shp_stage_batch / shp_run_staged): descriptor() + shp_stage_batch, then markStaged();
    // at the run, commitStaged() (or dropStaged() when the run failed)

    /** The open set's H2D is enqueued: it waits for its run, appends go to the other set (none is
     * free while two batches are staged: the caller runs the older one before the next append). */
    void markStaged() {
        staged.addLast(open);
        open = free.pollFirst();
    }

    int stagedCount() {
        return staged.size();
    }

    /** Rows of the oldest staged batch (the one shp_run_staged runs next). */
    long stagedSize() {
        return staged.isEmpty() ? 0 : staged.peekFirst().n;
    }

    /** The oldest staged batch ran: its rows join the history and its columns are the decoded ones
     * until the next append; the set is then free for appends.  Returns its first sequence number. */
    long commitStaged() {
        Columns c = staged.pollFirst();
        long first = commitRows(c);
        decoded = c;
        recycle(c);
        return first;
    }

    /** The oldest staged batch's run failed: the engine left its counter as before, so its rows are
     * dropped and the next staged batch takes its sequence numbers. */
    void dropStaged() {
        recycle(staged.pollFirst());
    }

    private void recycle(Columns c) {
        // its key / ts / stream columns stay readable through `decoded` until the next append (no
        // append runs while a flush decodes: both hold the runtime's lock)
        c.clear();
        if (open == null) {
            open = c;
        } else {
            free.addLast(c);
        }
    }

    int keyAt(long i) {
        return decoded.key.getAtIndex(JAVA_INT, i);
    }

    long tsAt(long i) {
        return decoded.ts.getAtIndex(JAVA_LONG, i);
    }

    int streamAt(long i) {
        return decoded.stream.getAtIndex(JAVA_INT, i);
    }

    /** Once the kept rows reach minTrim and have doubled since the last trim: ask the engine for its
     * oldest live sequence number (shp_engine_oldest_live_seq) and drop the rows below it. */
    void maybeTrim(LongSupplier oldestLive) {
        if (kept < trimAt) {
            return;
        }
        trim(oldestLive.getAsLong());
        trimAt = Math.max(minTrim, 2 * kept);
    }

    /** Drops every row below `lo`; a push partly below keeps its tail. */
    void trim(long lo) {
        while (head < history.size() && history.get(head).end() <= lo) {
            kept -= history.get(head).rows.length;
            history.set(head++, null);
        }
        if (head < history.size()) {
            Block b = history.get(head);
            if (b.seq0 < lo) {
                int cut = (int) (lo - b.seq0);
                history.set(head, new Block(lo, Arrays.copyOfRange(b.rows, cut, b.rows.length),
                        Arrays.copyOfRange(b.ts, cut, b.ts.length)));
                kept -= cut;
            }
        }
        if (head > 64 && head * 2 > history.size()) {  // drop the dead prefix, amortised
            history.subList(0, head).clear();
            head = 0;
        }
        floor = Math.max(floor, Math.min(lo, seq0));
    }

    /** The StreamEvent of sequence number `seq` (a match slot), rebuilt from the kept row, with the
     * before-window data the query's MetaStreamEvent expects for that stream. */
    StreamEvent event(long seq, int outputDataSize) {
        Block block = null;
        int last = history.size() - 1;
        if (last >= head && seq >= history.get(last).seq0) {   // the latest push: most matches name it
            block = seq < history.get(last).end() ? history.get(last) : null;
        } else {
            int lo = head;
            int hi = last;
            while (lo <= hi) {   // the last block with seq0 <= seq
                int mid = (lo + hi) >>> 1;
                if (history.get(mid).seq0 <= seq) {
                    lo = mid + 1;
                } else {
                    hi = mid - 1;
                }
            }
            if (hi >= head && seq < history.get(hi).end()) {
                block = history.get(hi);
            }
        }
        if (block == null) {
            // never expected: the engine names only rows at or after its oldest live one
            throw new IllegalStateException("event " + seq + " is not held (rows kept from " + floor + " to "
                    + seq0 + "): the engine named an event below its reported oldest live one");
        }
        int i = (int) (seq - block.seq0);
        StreamEvent e = new StreamEvent(0, 0, outputDataSize);
        e.setTimestamp(block.ts[i]);
        e.setOutputData(block.rows[i].clone());
        return e;
    }

    long nextSeq() {
        long n = open == null ? 0 : open.n;
        for (Columns c : staged) {
            n += c.n;
        }
        return seq0 + n;
    }

    // ---- snapshot support (GpuStateHolder): the rows the engine's state names travel with its blob,
    // as the reference's snapshot carries the StreamEvents of its partials

    /** The kept rows from `lo` on: {seqs (long[]), timestamps (long[]), data (Object[][])}. */
    Object[] liveRows(long lo) {
        List<Long> s = new ArrayList<>();
        List<Long> t = new ArrayList<>();
        List<Object[]> d = new ArrayList<>();
        for (int h = head; h < history.size(); h++) {
            Block b = history.get(h);
            for (int i = 0; i < b.rows.length; i++) {
                if (b.seq0 + i >= lo) {
                    s.add(b.seq0 + i);
                    t.add(b.ts[i]);
                    d.add(b.rows[i]);
                }
            }
        }
        long[] seqs = new long[s.size()];
        long[] tss = new long[t.size()];
        for (int i = 0; i < seqs.length; i++) {
            seqs[i] = s.get(i);
            tss[i] = t.get(i);
        }
        return new Object[]{seqs, tss, d.toArray(new Object[0][])};
    }

    /** After shp_restore: the history becomes the snapshot's rows (consecutive runs of sequence
     * numbers become blocks) and the next push starts at the engine's restored counter. */
    void restoreRows(long[] seqs, long[] tss, Object[][] data, long nextSeq) {
        history.clear();
        head = 0;
        kept = 0;
        int i = 0;
        while (i < seqs.length) {
            int j = i + 1;
            while (j < seqs.length && seqs[j] == seqs[j - 1] + 1) {
                j++;
            }
            history.add(new Block(seqs[i], Arrays.copyOfRange(data, i, j), Arrays.copyOfRange(tss, i, j)));
            kept += j - i;
            i = j;
        }
        if (!staged.isEmpty()) {
            throw new IllegalStateException("restore with staged batches: run them first");
        }
        discard();
        seq0 = nextSeq;
        floor = seqs.length > 0 ? seqs[0] : nextSeq;
        trimAt = Math.max(minTrim, 2 * kept);
    }
}
