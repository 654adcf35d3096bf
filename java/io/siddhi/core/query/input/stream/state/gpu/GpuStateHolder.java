/*
 * GpuStateHolder — hooks a GPU state query into SnapshotService (core/util/snapshot/
 * SnapshotService.java:90-188, restore :333) through the query's State
 * (core/util/snapshot/state/State.java:25-36), registered with
 * SiddhiQueryContext.generateStateHolder (core/config/SiddhiQueryContext.java:114-146).
 *
 * State.snapshot() returns the engine's blob (shp_snapshot) under "GpuEngineSnapshot" and, for
 * inspection and for tools that read the reference's key names, the same state decoded by
 * shp_snapshot_describe under "StateByKey": per partition key and state, the keys the reference's
 * processors snapshot — FirstEvent, PendingStateEventList, NewAndEveryStateEventList,
 * Initialized, Started (StreamPreStateProcessor.java:450-469), SuccessCondition /
 * StartStateReset (CountPreStateProcessor.java:206-219), IsActive, LastScheduledTime,
 * LastArrivalTime (AbsentStreamPreStateProcessor.java:328-341) and ToNotifyQueue
 * (Scheduler.java:349-360).  The rows the engine's partials name travel with the blob under
 * "LiveRows" (the reference's snapshot serialises the StreamEvents inside its partials; here they
 * are the ColumnarBatch rows from shp_engine_oldest_live_seq on), with "NextSeq" and, for CHAIN32,
 * the per-key rings.  restore() takes the blob, the rows and the rings back (the decoded form is
 * informational).
 * Source only: no JDK in this repository's image (DESIGN.md §6).
 */
package io.siddhi.core.query.input.stream.state.gpu;

import io.siddhi.core.util.snapshot.state.State;
import io.siddhi.core.util.snapshot.state.StateFactory;

import java.util.HashMap;
import java.util.Map;

public final class GpuStateHolder {

    private GpuStateHolder() {
    }

    public static StateFactory<State> factory(GpuStateStreamRuntime runtime) {
        return () -> new GpuState(runtime);
    }

    static final class GpuState extends State {
        private final GpuStateStreamRuntime runtime;

        GpuState(GpuStateStreamRuntime runtime) {
            this.runtime = runtime;
        }

        @Override
        public boolean canDestroy() {
            return false;
        }

        @Override
        public Map<String, Object> snapshot() {
            Map<String, Object> m = new HashMap<>();
            runtime.snapshotInto(m);
            return m;
        }

        @Override
        public void restore(Map<String, Object> state) {
            runtime.restoreFrom(state);
        }
    }
}
