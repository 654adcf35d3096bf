/*
 * GpuStateStreamRuntime — the drop-in StreamRuntime for a pattern / sequence query whose state
 * machine runs in libsiddhi_hip.so (SURVEY.md §8b, §8f-2).  Replaces StateStreamRuntime
 * (core/query/input/stream/state/StateStreamRuntime.java:38-98) and, below it, the
 * Stream/Count/Logical/Absent Pre/PostStateProcessor chain.  The Java host keeps SiddhiManager,
 * SiddhiAppRuntime, InputHandler.send, QuerySelector and the callbacks unchanged.
 *
 * Wiring (reference side):
 *   core/util/parser/InputStreamParser.java:88-93 — for a StateInputStream, return
 *     `GpuStateStreamRuntime.fromSiddhiQL(appText, queryName, ...)` instead of
 *     StateInputStreamParser.parseInputStream(...): the library lowers the query text itself
 *     (shp_engine_create_siddhiql; SHP_ERR_UNSUPPORTED = a construct outside the state path, and
 *     the host keeps the reference runtime for that query).
 *   core/util/SiddhiAppRuntimeBuilder.java:172-190 — unchanged: it subscribes the receivers
 *     getSingleStreamRuntimes() returns.  As the reference does, the runtime returns one
 *     SingleStreamRuntime per state, in MetaStateEvent order (StateInputStreamParser.java:86-125
 *     builds one ProcessStreamReceiver per stream id and StreamInnerStateRuntime.java:63-67 one
 *     SingleStreamRuntime per state on it), so QueryParserHelper.initStreamRuntime
 *     (core/util/parser/helper/QueryParserHelper.java:161-167) finds runtime i for state i; states
 *     of one stream share that stream's GpuStateReceiver, which StreamJunction.subscribe
 *     (core/stream/StreamJunction.java:334-338) subscribes once.
 *   Partitioned queries need no further change: the runtime IS a StateStreamRuntime, so
 *     PartitionParser.java:76 -> PartitionRuntimeImpl.addPartitionReceiver takes its
 *     `instanceof StateStreamRuntime` branch (core/partition/PartitionRuntimeImpl.java:243-258) and
 *     walks the query's state elements (:262-288) to create the outer streams'
 *     PartitionStreamReceivers; PartitionStreamReceiver.addStreamJunction (:291-310) subscribes
 *     runtime i's receiver (getSingleStreamRuntimes()) to the inner junction of its stream, and
 *     PartitionStreamReceiver.send (:262-272) sends each event under its partition key
 *     (SiddhiAppContext.startPartitionFlow), which GpuStateReceiver maps to a dense key id.  The
 *     per-key initPartition call (QueryRuntimeImpl.java:167-170) needs nothing: the engine creates
 *     a key's state on its first event.
 *   core/partition/PartitionStreamReceiver.java:176-283 — optional batching: append (key string,
 *     event) to the same batch instead of one send() per key run (GpuStateReceiver.append(ts, key,
 *     data), then endOfChunk()).
 *
 * Egress: every match reaches the QuerySelector inside its key's partition flow (emit():
 * SiddhiAppContext.startPartitionFlow(key) around selector.process, the caller's flow restored
 * after), as the reference emits them -- PartitionStreamReceiver.send (:262-272) for event matches,
 * the Scheduler's timer loop (core/util/Scheduler.java:88-97) for timer matches -- so the selector's
 * per-key state (PartitionStateHolder.getState, core/util/snapshot/state/PartitionStateHolder.java:
 * 43-48: aggregators, output rate limiters) is the match's key's even when one push carries many keys.
 *
 * Clock (queries with an absent state): the runtime registers a TimeChangeListener with the app's
 * TimestampGenerator, as the query's Scheduler does (Scheduler.java:71-103), so a playback send on
 * ANY stream and the @app:playback(idle.time) heartbeat (TimestampGeneratorImpl.java:105-121,
 * 165-185) reach the engine: SYNC fires the due timers at once (shp_advance_clock, before the event
 * that moved the clock), DEFERRED appends a clock-only row to the batch.  In live mode it keeps one
 * wall-clock wake-up on the app's ScheduledExecutorService at the engine's earliest due time
 * (shp_engine_next_due), as Scheduler.schedule / EventCaller.run do (:129-155, :287-326).
 *
 * Match records come back in the engine's compact layout (SHP_LAYOUT_COMPACT through
 * shp_push_batch_compact: PAIRS32 on the sweep path, CHAIN32 on the count-sequence path, FULL on
 * the others) and are decoded here against the batch's own rows; the rows are kept by sequence
 * number from shp_engine_oldest_live_seq on (ColumnarBatch).  The Python mirror of the decoding
 * and retention rules is siddhi_amd/history.py + runtime.py, tested in tests/test_retention.py.
 *
 * Concurrency: the reference serialises a query with synchronized(patternSyncObject)
 * (SingleProcessStreamReceiver.java:52); every entry point here takes `lock`.
 * Source only: no JDK in this repository's image, so it is not compiled here (DESIGN.md §6).
 */
package io.siddhi.core.query.input.stream.state.gpu;

import io.siddhi.core.config.SiddhiAppContext;
import io.siddhi.core.config.SiddhiQueryContext;
import io.siddhi.core.event.ComplexEvent;
import io.siddhi.core.event.ComplexEventChunk;
import io.siddhi.core.event.MetaComplexEvent;
import io.siddhi.core.event.state.MetaStateEvent;
import io.siddhi.core.event.state.StateEvent;
import io.siddhi.core.event.stream.MetaStreamEvent;
import io.siddhi.core.event.stream.StreamEvent;
import io.siddhi.core.exception.SiddhiAppCreationException;
import io.siddhi.core.exception.SiddhiAppRuntimeException;
import io.siddhi.core.query.input.stream.single.SingleStreamRuntime;
import io.siddhi.core.query.input.stream.state.StateStreamRuntime;
import io.siddhi.core.query.processor.ProcessingMode;
import io.siddhi.core.query.processor.Processor;
import io.siddhi.core.query.selector.QuerySelector;
import io.siddhi.query.api.definition.AbstractDefinition;
import io.siddhi.query.api.definition.Attribute;

import java.lang.foreign.Arena;
import java.lang.foreign.MemorySegment;
import java.util.ArrayList;
import java.util.Arrays;
import java.util.List;
import java.util.Map;
import java.util.concurrent.Executors;
import java.util.concurrent.ScheduledExecutorService;
import java.util.concurrent.ScheduledFuture;
import java.util.concurrent.TimeUnit;
import java.util.concurrent.locks.ReentrantLock;

import static java.lang.foreign.ValueLayout.ADDRESS;
import static java.lang.foreign.ValueLayout.JAVA_BYTE;
import static java.lang.foreign.ValueLayout.JAVA_INT;
import static java.lang.foreign.ValueLayout.JAVA_LONG;
import static java.lang.foreign.ValueLayout.JAVA_SHORT;

public final class GpuStateStreamRuntime extends StateStreamRuntime {

    /** When appended events reach the engine (and so when callbacks fire).
     * SYNC: at the end of every receive(...) call -- one push per InputHandler.send, callbacks
     *   fire before send returns, as in the reference (a send(Event[]) is one push).
     * DEFERRED: when the batch is full, every maxDelayMillis on a flusher thread, and before any
     *   point that observes state (advanceClock, snapshot, shutdown); callbacks then fire on the
     *   flusher (or the filling sender's) thread, as with an @async junction
     *   (core/stream/StreamJunction.java:101-131).  Synchronous single-event senders then share one
     *   push instead of paying a full push (sort, kernels, status read) per event.
     * PIPELINED: DEFERRED's flush points, with each flush staging its batch (shp_stage_batch: the H2D
     *   copies from page-locked columns on the engine's copy stream) and running the batch staged
     *   before it (shp_run_staged), so batch i+1's copies overlap batch i's kernels (bench.py
     *   end_to_end "pipelined").  A batch's callbacks fire one flush later; a flush with nothing new
     *   runs what is staged, and every point that observes state drains both first. */
    public enum FlushPolicy { SYNC, DEFERRED, PIPELINED }

    private final Arena arena = Arena.ofShared();
    private final ReentrantLock lock = new ReentrantLock();
    private final MemorySegment engine;            // shp_engine*
    private final MemorySegment matches;           // shp_matches, filled by the library
    private final ColumnarBatch batch;
    private final MetaStateEvent metaStateEvent;
    private final int numStates;
    private final int outputDataSize;
    private final List<SingleStreamRuntime> singleStreamRuntimes = new ArrayList<>();
    private final int layout;                      // the resolved SHP_LAYOUT_COMPACT: PAIRS32, CHAIN32 or FULL
    private final int maxKeys;
    private final int chainM;                      // CHAIN32: a chain's longest length (the count's max)
    private long[] ring;                           // CHAIN32: per key, its last chainM sequence numbers
    private int[] ringLen;
    private Processor selector;                    // QuerySelector (setCommonProcessor)
    private final NativeDictionary strings;        // string values, shared with the filters' constants
    private final NativeDictionary keys;           // partition keys, bounded by max_keys
    private final FlushPolicy policy;
    private final ScheduledExecutorService flusher;
    private final ScheduledFuture<?> flushTask;
    // DEFERRED: a push that failed on the flusher thread, rethrown to the next caller (append,
    // flush, advanceClock, snapshot) so the sender sees it; the flusher keeps running
    private volatile RuntimeException deferredFailure;
    private final boolean partitioned;             // matches are emitted inside their key's flow
    private final boolean timers;                  // an absent state: the query listens to the app clock
    private final SiddhiAppContext appContext;
    private ScheduledFuture<?> wake;               // live mode: the wall-clock wake-up at the next due time
    private long wakeAt = Long.MAX_VALUE;
    private volatile boolean closed;

    /**
     * The Java host's entry point: the library lowers the query from the app text
     * (shp_engine_create_siddhiql), so nothing on the Java side builds a program.
     *
     * @param appText    the SiddhiQL app (what SiddhiManager.createSiddhiAppRuntime was given)
     * @param queryName  the query's @info(name=...) (or "query<N>" by position in the app)
     */
    public static GpuStateStreamRuntime fromSiddhiQL(String appText, String queryName, int maxKeys, long maxBatch,
                                                     int device, long startClock, MetaStateEvent metaStateEvent,
                                                     Map<String, AbstractDefinition> streamDefinitionMap,
                                                     SiddhiQueryContext queryContext, FlushPolicy policy,
                                                     long maxDelayMillis) {
        NativeDictionary strings = new NativeDictionary(0, "string values");
        String program;
        try {
            program = ShpNative.compileSiddhiQL(appText, queryName, strings);
        } catch (IllegalArgumentException e) {
            strings.close();
            throw new SiddhiAppCreationException("shp_compile_siddhiql: " + e.getMessage(), e);
        }
        ProgramInfo info = ProgramInfo.parse(program);
        try {
            populateMeta(metaStateEvent, info, streamDefinitionMap);
            return new GpuStateStreamRuntime(appText, queryName, info, info.partitioned ? maxKeys : 1, maxBatch,
                    device, startClock, metaStateEvent, queryContext, strings, policy, maxDelayMillis);
        } catch (RuntimeException e) {
            strings.close();  // the constructor released everything else it had made
            throw e;
        }
    }

    /**
     * One MetaStreamEvent per state, in state order, as SingleInputStreamParser.parseInputStream /
     * initMetaStreamEvent (core/util/parser/SingleInputStreamParser.java:99-104, 261-296) add them
     * while StateInputStreamParser walks the state tree: the stream's definition, the state's
     * reference id when it differs from the stream id, multiValue for a count state.  Every
     * attribute of the definition is registered as output data in definition order, because the
     * match events are rebuilt from the rows as sent (ColumnarBatch.event); the selector's
     * variables (ExpressionParser.parseVariable, addOutputData) then resolve to those positions.
     * A MetaStateEvent that already holds the states (a host that ran the reference parser for
     * them) is left as it is.
     */
    static void populateMeta(MetaStateEvent meta, ProgramInfo info, Map<String, AbstractDefinition> defs) {
        int n = info.stateStream.length;
        if (meta.getStreamEventCount() == n) {
            return;
        }
        if (meta.getStreamEventCount() != 0) {
            throw new SiddhiAppCreationException("MetaStateEvent holds " + meta.getStreamEventCount()
                    + " stream events, the lowered query " + n + " states");
        }
        for (int st = 0; st < n; st++) {
            String streamId = info.streams[info.stateStream[st]];
            AbstractDefinition def = defs == null ? null : defs.get(streamId);
            if (def == null) {
                throw new SiddhiAppCreationException("Stream definition with ID '" + streamId + "' has not been defined");
            }
            MetaStreamEvent m = new MetaStreamEvent();
            m.addInputDefinition(def);
            String ref = info.stateRef[st];
            if (ref != null && !ref.equals(streamId)) {
                m.setInputReferenceId(ref);
            }
            m.setMultiValue(info.stateMulti[st]);
            for (Attribute a : def.getAttributeList()) {
                m.addOutputData(a);
            }
            meta.addEvent(m);
        }
    }

    /**
     * @param appText      the SiddhiQL app; the library lowers query `queryName` of it
     *                     (shp_engine_create_siddhiql), interning string constants in `strings`
     * @param info         the lowered program's streams, columns and per-state streams (ProgramInfo)
     * @param maxKeys      partition-key dictionary capacity (1 when the query is not partitioned)
     * @param maxBatch     events per push (a batch is flushed when full, on send return, or by timer)
     * @param device       HIP device ordinal
     * @param startClock   the event-time clock at start() (0 in playback mode)
     * On failure every native handle made here (engine, key dictionary) and the arena are released
     * before the exception leaves; `strings` stays the caller's.
     */
    GpuStateStreamRuntime(String appText, String queryName, ProgramInfo info, int maxKeys, long maxBatch, int device,
                          long startClock, MetaStateEvent metaStateEvent, SiddhiQueryContext queryContext,
                          NativeDictionary strings, FlushPolicy policy, long maxDelayMillis) {
        super(queryContext, metaStateEvent);
        this.metaStateEvent = metaStateEvent;
        this.maxKeys = maxKeys;
        this.chainM = Math.max(1, info.countMax);
        this.strings = strings;
        this.policy = policy;
        this.partitioned = info.partitioned;
        this.timers = info.timers;
        this.appContext = queryContext.getSiddhiAppContext();
        this.outputDataSize = metaStateEvent.getOutputDataAttributes() == null ? 0
                : metaStateEvent.getOutputDataAttributes().size();
        NativeDictionary keyDict = null;
        MemorySegment eng = MemorySegment.NULL;
        ColumnarBatch cb = null;
        try {
            keyDict = new NativeDictionary(maxKeys, "partition keys (max_keys = " + maxKeys + ")");
            MemorySegment cfg = arena.allocate(ShpNative.CONFIG);
            cfg.set(JAVA_INT, ShpNative.CFG_DEVICE, device);
            cfg.set(JAVA_INT, ShpNative.CFG_MAX_KEYS, maxKeys);
            cfg.set(JAVA_LONG, ShpNative.CFG_MAX_BATCH, maxBatch);
            cfg.set(JAVA_LONG, ShpNative.CFG_MAX_MATCHES, 0L);       // engine default
            cfg.set(JAVA_LONG, ShpNative.CFG_START_CLOCK, startClock);
            cfg.set(JAVA_INT, ShpNative.CFG_FORCE_GENERAL, 0);       // auto path
            cfg.set(JAVA_INT, ShpNative.CFG_PROFILE_KERNELS, 0);
            cfg.set(JAVA_INT, ShpNative.CFG_MATCH_LAYOUT, ShpNative.LAYOUT_COMPACT);
            MemorySegment out = arena.allocate(ADDRESS);
            int rc;
            try {
                rc = (int) ShpNative.ENGINE_CREATE_SIDDHIQL.invokeExact(arena.allocateFrom(appText),
                        queryName == null ? MemorySegment.NULL : arena.allocateFrom(queryName), strings.handle(), cfg,
                        out);
            } catch (Throwable t) {
                throw new SiddhiAppCreationException("shp_engine_create_siddhiql failed: " + t, t);
            }
            if (rc != ShpNative.OK) {
                // SHP_ERR_UNSUPPORTED = a construct outside the state path: the host falls back to
                // StateInputStreamParser (the reference runtime) for this query
                throw new SiddhiAppCreationException("shp_engine_create_siddhiql: " + ShpNative.codeName(rc));
            }
            eng = out.get(ADDRESS, 0);
            try {
                numStates = (int) ShpNative.NUM_STATES.invokeExact(eng);
            } catch (Throwable t) {
                throw new SiddhiAppCreationException("shp_engine_num_states failed", t);
            }
            if (numStates != metaStateEvent.getStreamEventCount() || numStates != info.stateStream.length) {
                throw new SiddhiAppCreationException("state count mismatch: engine " + numStates + ", MetaStateEvent "
                        + metaStateEvent.getStreamEventCount() + ", program " + info.stateStream.length);
            }
            // one receiver per stream id, one SingleStreamRuntime per state on its stream's receiver,
            // paired with that state's MetaStreamEvent (QueryParserHelper.java:161-167 indexes by state)
            GpuStateReceiver[] receivers = new GpuStateReceiver[info.streams.length];
            for (int st = 0; st < numStates; st++) {
                int s;
                try {
                    s = (int) ShpNative.STATE_STREAM.invokeExact(eng, st);
                } catch (Throwable t) {
                    throw new SiddhiAppCreationException("shp_engine_state_stream failed", t);
                }
                if (s < 0 || s >= receivers.length || s != info.stateStream[st]) {
                    throw new SiddhiAppCreationException("state " + st + ": engine stream " + s + ", program stream "
                            + info.stateStream[st]);
                }
                if (receivers[s] == null) {
                    receivers[s] = new GpuStateReceiver(info.streams[s], s, this, queryContext);
                }
                singleStreamRuntimes.add(new SingleStreamRuntime(receivers[s], null, ProcessingMode.BATCH,
                        metaStateEvent.getMetaStreamEvent(st)));
            }
            try (Arena a = Arena.ofConfined()) {
                layout = (int) (long) ShpNative.ENGINE_STAT.invokeExact(eng, a.allocateFrom("match_layout"));
            } catch (Throwable t) {
                throw new SiddhiAppCreationException("shp_engine_stat failed", t);
            }
            matches = arena.allocate(ShpNative.MATCHES);
            // PIPELINED with 2-byte key ids possible: the narrow form's columns too (10 B/event for one
            // 4-byte column instead of 16; bench.py end_to_end "pipelined_narrow")
            cb = new ColumnarBatch(arena, maxBatch, info.columns, strings, 1 << 12,
                    policy == FlushPolicy.PIPELINED ? 2 : 1, policy == FlushPolicy.PIPELINED && maxKeys <= 65536);
            if (policy == FlushPolicy.PIPELINED) {
                try {
                    cb.pin();
                } catch (Throwable t) {
                    throw new SiddhiAppCreationException("shp_host_register of the batch columns failed: " + t, t);
                }
            }
        } catch (RuntimeException e) {
            if (cb != null) {
                try {
                    cb.unpin();
                } catch (Throwable ignored) {
                    // the creation error is the one to report
                }
            }
            if (!eng.equals(MemorySegment.NULL)) {
                try {
                    ShpNative.ENGINE_DESTROY.invokeExact(eng);
                } catch (Throwable ignored) {
                    // the creation error is the one to report
                }
            }
            if (keyDict != null) {
                keyDict.close();
            }
            arena.close();
            throw e;
        }
        this.engine = eng;
        this.keys = keyDict;
        this.batch = cb;
        if (policy != FlushPolicy.SYNC) {
            flusher = Executors.newSingleThreadScheduledExecutor(r -> {
                Thread t = new Thread(r, "siddhi-gpu-flush");
                t.setDaemon(true);
                return t;
            });
            long d = Math.max(1, maxDelayMillis);
            // a failing push must not cancel the periodic task (ScheduledExecutorService suppresses
            // every later run after an exception): keep it, hand it to the next caller
            flushTask = flusher.scheduleWithFixedDelay(() -> {
                try {
                    flush();
                } catch (RuntimeException e) {
                    deferredFailure = e;
                }
            }, d, d, TimeUnit.MILLISECONDS);
        } else {
            flusher = null;
            flushTask = null;
        }
        if (timers) {
            // Scheduler.java:71-72: the query hears every move of the app clock -- a playback send
            // on any stream (InputHandler.java:59-92) and the idle.time heartbeat
            appContext.getTimestampGenerator().addTimeChangeListener(this::onTimeChange);
        }
    }

    /** A push that failed on the flusher thread (DEFERRED): thrown to the caller that comes next. */
    private void rethrowDeferred() {
        RuntimeException e = deferredFailure;
        if (e != null) {
            deferredFailure = null;
            throw new SiddhiAppRuntimeException("a deferred push failed (its events were dropped): " + e.getMessage(),
                    e);
        }
    }

    /** Dense id of a partition key string (the key of the current partition flow). */
    int keyId(String key) {
        return keys.id(key);
    }

    /** A receive(...) call returned: SYNC pushes now (callbacks before InputHandler.send returns). */
    void endOfReceive() {
        if (policy == FlushPolicy.SYNC) {
            flush();
        }
    }

    // ---------------------------------------------------------------- StateStreamRuntime
    @Override
    public List<SingleStreamRuntime> getSingleStreamRuntimes() {
        return singleStreamRuntimes;
    }

    @Override
    public void setCommonProcessor(Processor commonProcessor) {
        this.selector = commonProcessor;
    }

    @Override
    public MetaComplexEvent getMetaComplexEvent() {
        return metaStateEvent;
    }

    @Override
    public ProcessingMode getProcessingMode() {
        return ProcessingMode.BATCH;
    }

    @Override
    public QuerySelector getQuerySelector() {
        return null;
    }

    /** Called by the Sequence receivers after each event (SequenceSingleProcessStreamReceiver.java:43,
     * SequenceMultiProcessStreamReceiver.java:49), which GpuStateReceiver replaces: the engine resets
     * and updates its states per event itself. */
    @Override
    public void resetAndUpdate() {
    }

    /** QueryRuntimeImpl.initPartition (:167-170) for a new partition key (PartitionStreamReceiver.send
     * :266): the engine creates a key's state -- the start partials and, for absent states, the
     * partitionCreated timers -- at the key's first event, so nothing happens here. */
    @Override
    public void initPartition() {
    }

    // ---------------------------------------------------------------- ingress (GpuStateReceiver)
    void append(long timestamp, int keyId, int streamIndex, Object[] data) {
        rethrowDeferred();
        lock.lock();
        try {
            batch.append(timestamp, keyId, streamIndex, data);
            if (batch.full()) {
                flush();
            }
        } finally {
            lock.unlock();
        }
    }

    /** One shp_push_batch of the appended events, then one StateEvent per match into the
     * selector, in record order (per key = the reference's emission order).  PIPELINED: stage the
     * appended events, then run the batch staged before them (or, with nothing new, what is staged). */
    void flush() {
        lock.lock();
        try {
            if (policy == FlushPolicy.PIPELINED) {
                boolean fresh = stageOpen();
                if (batch.stagedCount() > (fresh ? 1 : 0)) {
                    runStaged();
                }
                return;
            }
            if (batch.size() == 0) {
                return;
            }
            int rc;
            long pushed = batch.size();
            try {
                rc = (int) ShpNative.PUSH_BATCH_COMPACT.invokeExact(engine, batch.descriptor(), matches);
            } catch (Throwable t) {
                batch.discard();
                throw new SiddhiAppRuntimeException("shp_push_batch failed: " + t, t);
            }
            if (rc != ShpNative.OK) {
                // the engine left its state (and its sequence counter) as before the push: drop the
                // rows without advancing the batch's seq0, so later matches keep resolving to the
                // right rows
                batch.discard();
                throw new SiddhiAppRuntimeException("shp_push_batch: " + ShpNative.codeName(rc) + ": "
                        + ShpNative.lastError(engine));
            }
            long seq0 = batch.commit();
            deliver(seq0, pushed);
            batch.maybeTrim(this::oldestLiveSeq);
            scheduleWake();
        } finally {
            lock.unlock();
        }
    }

    /** Every appended and staged event through the engine (PIPELINED's drain before the clock moves,
     * a snapshot or restore, shutdown); flush() otherwise. */
    private void drain() {
        lock.lock();
        try {
            flush();
            while (batch.stagedCount() > 0) {
                runStaged();
            }
        } finally {
            lock.unlock();
        }
    }

    /** PIPELINED: shp_stage_batch of the open rows (false when there are none). */
    private boolean stageOpen() {
        if (batch.size() == 0) {
            return false;
        }
        int rc;
        try {
            if (batch.narrowOk()) {   // ts offsets from the batch's first ts and 2-byte key ids
                rc = (int) ShpNative.STAGE_BATCH_NARROW.invokeExact(engine, batch.descriptor(), batch.narrowBase(),
                        batch.ts32(), batch.key16());
            } else {
                rc = (int) ShpNative.STAGE_BATCH.invokeExact(engine, batch.descriptor());
            }
        } catch (Throwable t) {
            batch.discard();
            throw new SiddhiAppRuntimeException("shp_stage_batch failed: " + t, t);
        }
        if (rc != ShpNative.OK) {
            batch.discard();   // not staged: the engine's counter and slots are as before
            throw new SiddhiAppRuntimeException("shp_stage_batch: " + ShpNative.codeName(rc) + ": "
                    + ShpNative.lastError(engine));
        }
        batch.markStaged();
        return true;
    }

    /** PIPELINED: shp_run_staged of the oldest staged batch, then its records as a push's. */
    private void runStaged() {
        long pushed = batch.stagedSize();
        int rc;
        try {
            rc = (int) ShpNative.RUN_STAGED.invokeExact(engine, matches);
        } catch (Throwable t) {
            batch.dropStaged();
            throw new SiddhiAppRuntimeException("shp_run_staged failed: " + t, t);
        }
        if (rc != ShpNative.OK) {
            batch.dropStaged();   // as a failed push: the engine's state and counter are as before
            throw new SiddhiAppRuntimeException("shp_run_staged: " + ShpNative.codeName(rc) + ": "
                    + ShpNative.lastError(engine));
        }
        long seq0 = batch.commitStaged();
        deliver(seq0, pushed);
        batch.maybeTrim(this::oldestLiveSeq);
        scheduleWake();
    }

    /** shp_engine_oldest_live_seq: the oldest event an open partial of the committed state holds. */
    private long oldestLiveSeq() {
        try (Arena a = Arena.ofConfined()) {
            MemorySegment out = a.allocate(JAVA_LONG);
            int rc = (int) ShpNative.OLDEST_LIVE_SEQ.invokeExact(engine, out);
            if (rc != ShpNative.OK) {
                throw new SiddhiAppRuntimeException("shp_engine_oldest_live_seq: " + ShpNative.lastError(engine));
            }
            return out.get(JAVA_LONG, 0);
        } catch (RuntimeException e) {
            throw e;
        } catch (Throwable t) {
            throw new SiddhiAppRuntimeException("shp_engine_oldest_live_seq failed: " + t, t);
        }
    }

    /** The query's TimeChangeListener (Scheduler.java:71-103): the app clock moved to `now` -- a
     * playback send on any stream (before its event reaches a receiver) or the idle heartbeat.  SYNC
     * fires the timers due by `now` at once, as the Scheduler does inside onTimeChange; DEFERRED adds
     * a clock-only row to the batch (absorbed by the event that follows when the send is this
     * query's, ColumnarBatch.append), and its timer matches come with the push. */
    void onTimeChange(long now) {
        if (closed) {
            return;
        }
        if (policy == FlushPolicy.SYNC) {
            advanceClock(now);
            return;
        }
        rethrowDeferred();
        lock.lock();
        try {
            batch.appendClock(now);
            if (batch.full()) {
                flush();
            }
        } finally {
            lock.unlock();
        }
    }

    /** shp_engine_next_due: the earliest head of any key's timer queue, Long.MAX_VALUE when none. */
    private long nextDue() {
        try (Arena a = Arena.ofConfined()) {
            MemorySegment out = a.allocate(JAVA_LONG);
            int rc = (int) ShpNative.NEXT_DUE.invokeExact(engine, out);
            if (rc < 0) {
                throw new SiddhiAppRuntimeException("shp_engine_next_due: " + ShpNative.lastError(engine));
            }
            return rc == 1 ? out.get(JAVA_LONG, 0) : Long.MAX_VALUE;
        } catch (RuntimeException e) {
            throw e;
        } catch (Throwable t) {
            throw new SiddhiAppRuntimeException("shp_engine_next_due failed: " + t, t);
        }
    }

    /** Live mode (not playback): keep one wake-up on the app's ScheduledExecutorService at the
     * engine's earliest due time, as Scheduler.schedule arms the EventCaller for a queue head
     * (Scheduler.java:129-155) and EventCaller.run re-arms for the next (:287-326).  The wake-up
     * advances the engine to the wall clock, which fires every timer due by then.  Called under
     * `lock` after every push. */
    private void scheduleWake() {
        if (!timers || closed || appContext.isPlayback()) {
            return;
        }
        long due = nextDue();
        if (due == Long.MAX_VALUE || (wake != null && !wake.isDone() && wakeAt <= due)) {
            return;
        }
        if (wake != null) {
            wake.cancel(false);
        }
        wakeAt = due;
        long delay = Math.max(0, due - appContext.getTimestampGenerator().currentTime());
        wake = appContext.getScheduledExecutorService().schedule(this::onWake, delay, TimeUnit.MILLISECONDS);
    }

    private void onWake() {
        lock.lock();
        try {
            wake = null;               // this wake-up has run: advanceClock arms the next one
            wakeAt = Long.MAX_VALUE;
        } finally {
            lock.unlock();
        }
        try {
            if (!closed && !appContext.isPlayback()) {
                advanceClock(appContext.getTimestampGenerator().currentTime());
            }
        } catch (RuntimeException e) {
            deferredFailure = e;       // no caller on the executor's thread: the next one sees it
        }
    }

    /** TimestampGeneratorImpl.setCurrentTimestamp with no event (absent-state timers). */
    void advanceClock(long now) {
        rethrowDeferred();
        lock.lock();
        try {
            drain();
            int rc;
            try {
                rc = (int) ShpNative.ADVANCE_CLOCK.invokeExact(engine, now, matches);
            } catch (Throwable t) {
                throw new SiddhiAppRuntimeException("shp_advance_clock failed: " + t, t);
            }
            if (rc != ShpNative.OK) {
                throw new SiddhiAppRuntimeException("shp_advance_clock: " + ShpNative.lastError(engine));
            }
            deliverFull();   // a clock-only event: FULL records (timer matches), no new rows
            scheduleWake();
        } finally {
            lock.unlock();
        }
    }

    /** One match into the QuerySelector, inside its key's partition flow (the only call of
     * selector.process): PartitionStreamReceiver.send (:262-272) runs event matches under
     * SiddhiAppContext.startPartitionFlow(key) and the Scheduler timer matches the same way
     * (Scheduler.java:88-97), so the selector's per-key state is looked up under the match's key.
     * The caller's flow (a sender's PartitionStreamReceiver.send of another key, in a batched push
     * or when key A's timer fires on key B's event) is restored after it. */
    private void emit(int keyId, StateEvent se) {
        if (!partitioned) {
            selector.process(new ComplexEventChunk<>(se, se));
            return;
        }
        String prev = SiddhiAppContext.getPartitionFlowId();
        SiddhiAppContext.startPartitionFlow(keys.string(keyId));
        try {
            selector.process(new ComplexEventChunk<>(se, se));
        } finally {
            if (prev == null) {
                SiddhiAppContext.stopPartitionFlow();
            } else {
                SiddhiAppContext.startPartitionFlow(prev);
            }
        }
    }

    /** The records of the push whose rows start at seq0 (pushed rows, still in the batch columns). */
    private void deliver(long seq0, long pushed) {
        int lay = ShpNative.matchesInt(matches, "layout");
        if (lay == ShpNative.LAYOUT_PAIRS32) {
            deliverPairs32(seq0);
        } else if (lay == ShpNative.LAYOUT_CHAIN32) {
            deliverChain32(seq0, pushed);
        } else {
            deliverFull();
        }
    }

    /** PAIRS32 (sweep path, 2 states): word pair (e2's batch index, e2 seq - e1 seq).  The engine
     * writes them per key in emission order, across keys in owner order; the reference emits at
     * e2's arrival, so they are ordered stably by e2's index (history.decode_pairs32). */
    private void deliverPairs32(long seq0) {
        long m = ShpNative.matchesLong(matches, "m");
        if (m == 0) {
            return;
        }
        MemorySegment w = ShpNative.matchesPtr(matches, "refs", m * 8);
        long[] order = new long[(int) m];
        for (int j = 0; j < m; j++) {
            order[j] = (Integer.toUnsignedLong(w.getAtIndex(JAVA_INT, 2L * j)) << 32) | j;
        }
        Arrays.sort(order);   // by e2's index, then the engine's order (stable)
        int out0 = metaStateEvent.getMetaStreamEvent(0).getOutputData().size();
        int out1 = metaStateEvent.getMetaStreamEvent(1).getOutputData().size();
        for (long o : order) {
            int j = (int) (o & 0xffffffffL);
            long idx = o >>> 32;
            long e2 = seq0 + idx;
            long e1 = e2 - Integer.toUnsignedLong(w.getAtIndex(JAVA_INT, 2L * j + 1));
            StateEvent se = new StateEvent(numStates, outputDataSize);
            se.setTimestamp(batch.tsAt(idx));
            se.setType(ComplexEvent.Type.CURRENT);
            se.addEvent(0, batch.event(e1, out0));
            se.addEvent(1, batch.event(e2, out1));
            emit(batch.keyAt(idx), se);
        }
    }

    /** CHAIN32 (count-sequence path `e1=S[..]<1:M>, e2=S[..]`): word = e2's batch index | L << 28; e1's
     * chain is the L events of e2's key just before e2.  The pushed rows are walked in order with a
     * ring of each key's last M sequence numbers (history.ChainRings); a sequence emits at most one
     * match per event, at that event, so batch order is the reference's emission order. */
    private void deliverChain32(long seq0, long pushed) {
        long m = ShpNative.matchesLong(matches, "m");
        if (ring == null) {
            ring = new long[maxKeys * chainM];
            ringLen = new int[maxKeys];
        }
        int[] lenAt = null;
        if (m > 0) {
            MemorySegment w = ShpNative.matchesPtr(matches, "refs", m * 4);
            lenAt = new int[(int) pushed];
            Arrays.fill(lenAt, -1);
            for (long j = 0; j < m; j++) {
                int x = w.getAtIndex(JAVA_INT, j);
                lenAt[x & 0x0FFFFFFF] = x >>> 28;
            }
        }
        int out0 = metaStateEvent.getMetaStreamEvent(0).getOutputData().size();
        int out1 = metaStateEvent.getMetaStreamEvent(1).getOutputData().size();
        for (int i = 0; i < pushed; i++) {
            if (batch.streamAt(i) < 0) {
                continue;   // a clock-only row is no key's event
            }
            int k = batch.keyAt(i);
            int base = k * chainM;
            int have = ringLen[k];
            if (lenAt != null && lenAt[i] >= 0) {
                int len = lenAt[i];
                if (len > have) {
                    throw new SiddhiAppRuntimeException("CHAIN32: a chain of " + len + " events before row " + i
                            + " but key " + k + " holds " + have);
                }
                StateEvent se = new StateEvent(numStates, outputDataSize);
                se.setTimestamp(batch.tsAt(i));
                se.setType(ComplexEvent.Type.CURRENT);
                for (int t = have - len; t < have; t++) {
                    se.addEvent(0, batch.event(ring[base + t], out0));   // the count state's chain, in order
                }
                se.addEvent(1, batch.event(seq0 + i, out1));
                emit(k, se);
            }
            if (have == chainM) {
                System.arraycopy(ring, base + 1, ring, base, chainM - 1);
                have--;
            }
            ring[base + have] = seq0 + i;
            ringLen[k] = have + 1;
        }
    }

    // StateEvents from FULL records: slot s of match i holds slot_len[i*S+s] event sequence
    // numbers from refs[ref_off[i] + ...] (a count state's chain, in order); -1 = an empty slot
    private void deliverFull() {
        long m = ShpNative.matchesLong(matches, "m");
        if (m == 0) {
            return;
        }
        MemorySegment key = ShpNative.matchesPtr(matches, "key", m * 4);
        MemorySegment ts = ShpNative.matchesPtr(matches, "ts", m * 8);
        MemorySegment type = ShpNative.matchesPtr(matches, "type", m);
        MemorySegment refOff = ShpNative.matchesPtr(matches, "ref_off", m * 8);
        MemorySegment slotLen = ShpNative.matchesPtr(matches, "slot_len", m * numStates * 2L);
        long nrefs = 0;
        for (long i = 0; i < m * numStates; i++) {
            nrefs += slotLen.getAtIndex(JAVA_SHORT, i);
        }
        MemorySegment refs = ShpNative.matchesPtr(matches, "refs", Math.max(1, nrefs) * 8);
        for (long i = 0; i < m; i++) {
            StateEvent se = new StateEvent(numStates, outputDataSize);
            se.setTimestamp(ts.getAtIndex(JAVA_LONG, i));
            se.setType(type.get(JAVA_BYTE, i) == 0 ? ComplexEvent.Type.CURRENT : ComplexEvent.Type.EXPIRED);
            long r = refOff.getAtIndex(JAVA_LONG, i);
            for (int s = 0; s < numStates; s++) {
                int len = slotLen.getAtIndex(JAVA_SHORT, i * numStates + s);
                for (int k = 0; k < len; k++) {
                    long seq = refs.getAtIndex(JAVA_LONG, r++);
                    if (seq >= 0) {
                        StreamEvent e = batch.event(seq,
                                metaStateEvent.getMetaStreamEvent(s).getOutputData().size());
                        se.addEvent(s, e);   // count states: a `next` chain, as StateEvent.addEvent builds it
                    }
                }
            }
            emit(key.getAtIndex(JAVA_INT, i), se);
        }
    }

    // ---------------------------------------------------------------- snapshot (GpuStateHolder)
    byte[] snapshot() {
        rethrowDeferred();
        lock.lock();
        try {
            drain();
            MemorySegment buf = arena.allocate(ADDRESS);
            MemorySegment len = arena.allocate(JAVA_LONG);
            int rc = (int) ShpNative.SNAPSHOT.invokeExact(engine, buf, len);
            if (rc != ShpNative.OK) {
                throw new SiddhiAppRuntimeException("shp_snapshot: " + ShpNative.lastError(engine));
            }
            long n = len.get(JAVA_LONG, 0);
            return buf.get(ADDRESS, 0).reinterpret(n).toArray(JAVA_BYTE);
        } catch (RuntimeException e) {
            throw e;
        } catch (Throwable t) {
            throw new SiddhiAppRuntimeException("shp_snapshot failed: " + t, t);
        } finally {
            lock.unlock();
        }
    }

    /** The snapshot in the reference's State.snapshot() key names (shp_snapshot_describe, JSON):
     * per key and state, FirstEvent / PendingStateEventList / NewAndEveryStateEventList /
     * Initialized / Started (StreamPreStateProcessor.java:450-469), plus IsActive /
     * LastScheduledTime / LastArrivalTime for absent states and ToNotifyQueue for timers. */
    String describe(byte[] blob) {
        try (Arena a = Arena.ofConfined()) {
            MemorySegment in = a.allocateFrom(JAVA_BYTE, blob);
            long need = (long) ShpNative.SNAPSHOT_DESCRIBE.invokeExact(engine, in, (long) blob.length,
                    MemorySegment.NULL, 0L);
            if (need < 0) {
                throw new SiddhiAppRuntimeException("shp_snapshot_describe: " + ShpNative.codeName((int) need));
            }
            MemorySegment out = a.allocate(need + 1);
            long got = (long) ShpNative.SNAPSHOT_DESCRIBE.invokeExact(engine, in, (long) blob.length, out, need + 1);
            return out.getString(0);
        } catch (RuntimeException e) {
            throw e;
        } catch (Throwable t) {
            throw new SiddhiAppRuntimeException("shp_snapshot_describe failed: " + t, t);
        }
    }

    /** State.snapshot() for GpuStateHolder: the engine blob, the rows its partials name (the reference's
     * snapshot carries those StreamEvents inside its partials) and, for CHAIN32, the per-key rings. */
    void snapshotInto(Map<String, Object> m) {
        lock.lock();
        try {
            byte[] blob = snapshot();
            m.put("GpuEngineSnapshot", blob);
            m.put("StateByKey", describe(blob));
            m.put("LiveRows", batch.liveRows(oldestLiveSeq()));
            m.put("NextSeq", batch.nextSeq());
            if (ring != null) {
                m.put("ChainRings", new Object[]{ring.clone(), ringLen.clone()});
            }
        } finally {
            lock.unlock();
        }
    }

    /** State.restore(): the engine blob, then the rows and rings that travelled with it.  A state
     * without the rows (a snapshot of an older build: GpuEngineSnapshot / StateByKey only) is refused
     * before the engine is touched, so engine and row history never disagree. */
    void restoreFrom(Map<String, Object> m) {
        if (!(m.get("GpuEngineSnapshot") instanceof byte[]) || !(m.get("LiveRows") instanceof Object[])
                || !(m.get("NextSeq") instanceof Long)) {
            throw new SiddhiAppRuntimeException("GPU state snapshot without GpuEngineSnapshot / LiveRows / NextSeq "
                    + "(taken by an older build?): the rows its partials name are missing, not restored");
        }
        lock.lock();
        try {
            while (batch.stagedCount() > 0) {
                runStaged();   // PIPELINED: staged events were sent before the restore
            }
            restore((byte[]) m.get("GpuEngineSnapshot"));
            Object[] rows = (Object[]) m.get("LiveRows");
            batch.restoreRows((long[]) rows[0], (long[]) rows[1], (Object[][]) rows[2], (Long) m.get("NextSeq"));
            Object[] rings = (Object[]) m.get("ChainRings");
            if (rings != null) {
                ring = ((long[]) rings[0]).clone();
                ringLen = ((int[]) rings[1]).clone();
            } else {
                ring = null;
                ringLen = null;
            }
        } finally {
            lock.unlock();
        }
    }

    void restore(byte[] blob) {
        lock.lock();
        try (Arena a = Arena.ofConfined()) {
            MemorySegment in = a.allocateFrom(JAVA_BYTE, blob);
            int rc = (int) ShpNative.RESTORE.invokeExact(engine, in, (long) blob.length);
            if (rc != ShpNative.OK) {
                throw new SiddhiAppRuntimeException("shp_restore: " + ShpNative.lastError(engine));
            }
        } catch (RuntimeException e) {
            throw e;
        } catch (Throwable t) {
            throw new SiddhiAppRuntimeException("shp_restore failed: " + t, t);
        } finally {
            lock.unlock();
        }
    }

    /** SiddhiAppRuntime.shutdown for the query. */
    public void shutdown() {
        closed = true;                 // the app clock's listener and the wake-up become no-ops
        lock.lock();
        try {
            if (wake != null) {
                wake.cancel(false);
            }
        } finally {
            lock.unlock();
        }
        if (flushTask != null) {
            flushTask.cancel(false);
            flusher.shutdown();
        }
        lock.lock();
        try {
            drain();
            ShpNative.ENGINE_DESTROY.invokeExact(engine);
            batch.unpin();
            keys.close();
            strings.close();
        } catch (Throwable t) {
            throw new SiddhiAppRuntimeException("shp_engine_destroy failed: " + t, t);
        } finally {
            lock.unlock();
            arena.close();
        }
    }
}
