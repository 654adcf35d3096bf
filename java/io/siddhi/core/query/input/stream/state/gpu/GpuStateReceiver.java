/*
 * GpuStateReceiver — what SiddhiAppRuntimeBuilder.addQuery (core/util/SiddhiAppRuntimeBuilder.java:
 * 172-190) subscribes to a stream's junction for a GPU state query.  Replaces the
 * Pattern/Sequence{Single,Multi}ProcessStreamReceivers (core/query/input/stream/state/receiver/*):
 * instead of running the processor chain per event under synchronized(patternSyncObject), each
 * receive appends the event to the runtime's columnar batch; a synchronous send flushes on return,
 * so callbacks fire before InputHandler.send returns, as in the reference.
 * Source only: no JDK in this repository's image (DESIGN.md §6).
 */
package io.siddhi.core.query.input.stream.state.gpu;

import io.siddhi.core.config.SiddhiQueryContext;
import io.siddhi.core.event.ComplexEvent;
import io.siddhi.core.event.Event;
import io.siddhi.core.query.input.ProcessStreamReceiver;

import java.util.List;

public final class GpuStateReceiver extends ProcessStreamReceiver {

    private final int streamIndex;
    private final GpuStateStreamRuntime runtime;
    private final SiddhiQueryContext queryContext;

    GpuStateReceiver(String streamId, int streamIndex, GpuStateStreamRuntime runtime,
                     SiddhiQueryContext queryContext) {
        super(streamId, queryContext);
        this.streamIndex = streamIndex;
        this.runtime = runtime;
        this.queryContext = queryContext;
    }

    /** Partition key dictionary id of the current flow: PartitionStreamReceiver.send sets the key
     * (SiddhiAppContext.startPartitionFlow, ValuePartitionExecutor.execute(...).toString()); the
     * host maps the string to a dense id (0 when not partitioned). */
    private int keyId() {
        String key = queryContext.getSiddhiAppContext().getPartitionFlowId();
        return key == null ? 0 : PartitionKeys.id(key);
    }

    @Override
    public void receive(ComplexEvent complexEvent) {
        for (ComplexEvent e = complexEvent; e != null; e = e.getNext()) {
            runtime.append(e.getTimestamp(), keyId(), streamIndex, e.getOutputData());
        }
        runtime.flush();
    }

    @Override
    public void receive(Event event) {
        runtime.append(event.getTimestamp(), keyId(), streamIndex, event.getData());
        runtime.flush();
    }

    @Override
    public void receive(Event[] events) {
        for (Event e : events) {
            runtime.append(e.getTimestamp(), keyId(), streamIndex, e.getData());
        }
        runtime.flush();
    }

    @Override
    public void receive(List<Event> events) {
        for (Event e : events) {
            runtime.append(e.getTimestamp(), keyId(), streamIndex, e.getData());
        }
        runtime.flush();
    }

    @Override
    public void receive(long timestamp, Object[] data) {
        runtime.append(timestamp, keyId(), streamIndex, data);
        runtime.flush();
    }

    /** The partitioned path batched (PartitionStreamReceiver.java:176-216 appends here instead of
     * one send() per key; the caller flushes once per incoming chunk). */
    public void append(long timestamp, int keyId, Object[] data) {
        runtime.append(timestamp, keyId, streamIndex, data);
    }

    public void flush() {
        runtime.flush();
    }

    /** Dense partition-key ids (the engine's cfg.max_keys bounds them). */
    static final class PartitionKeys {
        private static final java.util.concurrent.ConcurrentHashMap<String, Integer> IDS =
                new java.util.concurrent.ConcurrentHashMap<>();

        static int id(String key) {
            return IDS.computeIfAbsent(key, k -> IDS.size());
        }
    }
}
