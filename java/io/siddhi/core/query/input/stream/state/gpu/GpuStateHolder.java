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
 * (Scheduler.java:349-360).  restore() takes the blob back (the decoded form is informational).
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
            byte[] blob = runtime.snapshot();
            Map<String, Object> m = new HashMap<>();
            m.put("GpuEngineSnapshot", blob);
            m.put("StateByKey", runtime.describe(blob));
            return m;
        }

        @Override
        public void restore(Map<String, Object> state) {
            runtime.restore((byte[]) state.get("GpuEngineSnapshot"));
        }
    }
}
