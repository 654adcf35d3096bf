/*
 * GpuStateReceiver — what SiddhiAppRuntimeBuilder.addQuery (core/util/SiddhiAppRuntimeBuilder.java:
 * 172-190) subscribes to a stream's junction for a GPU state query.  Replaces the
 * Pattern/Sequence{Single,Multi}ProcessStreamReceivers (core/query/input/stream/state/receiver/*):
 * instead of running the processor chain per event under synchronized(patternSyncObject), each
 * receive appends the event to the runtime's columnar batch.  Under FlushPolicy.SYNC the batch is
 * pushed when the receive call returns (callbacks fire before InputHandler.send returns, as in the
 * reference; a send(Event[]) is one push); under DEFERRED it is pushed when full or by the
 * runtime's flusher (GpuStateStreamRuntime.FlushPolicy).
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
        return key == null ? 0 : runtime.keyId(key);
    }

    @Override
    public void receive(ComplexEvent complexEvent) {
        for (ComplexEvent e = complexEvent; e != null; e = e.getNext()) {
            runtime.append(e.getTimestamp(), keyId(), streamIndex, e.getOutputData());
        }
        runtime.endOfReceive();
    }

    @Override
    public void receive(Event event) {
        runtime.append(event.getTimestamp(), keyId(), streamIndex, event.getData());
        runtime.endOfReceive();
    }

    @Override
    public void receive(Event[] events) {
        for (Event e : events) {
            runtime.append(e.getTimestamp(), keyId(), streamIndex, e.getData());
        }
        runtime.endOfReceive();
    }

    @Override
    public void receive(List<Event> events) {
        for (Event e : events) {
            runtime.append(e.getTimestamp(), keyId(), streamIndex, e.getData());
        }
        runtime.endOfReceive();
    }

    @Override
    public void receive(long timestamp, Object[] data) {
        runtime.append(timestamp, keyId(), streamIndex, data);
        runtime.endOfReceive();
    }

    /** The partitioned path batched (PartitionStreamReceiver.java:176-216 appends here instead of
     * one send() per key; the caller calls endOfChunk() once per incoming chunk).  key: the
     * partition key string (ValuePartitionExecutor.execute(...).toString()), mapped to a dense id
     * by the runtime's own bounded dictionary (one per query runtime, not JVM-wide). */
    public void append(long timestamp, String key, Object[] data) {
        runtime.append(timestamp, key == null ? 0 : runtime.keyId(key), streamIndex, data);
    }

    public void endOfChunk() {
        runtime.endOfReceive();
    }
}
