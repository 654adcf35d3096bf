/*
 * siddhi_hip.h — C-ABI of libsiddhi_hip.so, the MI355X engine for Siddhi's
 * pattern/sequence path (io.siddhi.core.query.input.stream.state).
 *
 * Drop-in boundary. The reference has no plugin SPI for state
 * runtimes: a StateStreamRuntime is built at
 *   modules/siddhi-core/src/main/java/io/siddhi/core/util/parser/InputStreamParser.java:88-93
 * and fed through StreamJunction.Receiver.receive(...)
 *   modules/siddhi-core/src/main/java/io/siddhi/core/stream/StreamJunction.java:443-456
 * by the Pattern/Sequence{Single,Multi}ProcessStreamReceivers
 *   modules/siddhi-core/src/main/java/io/siddhi/core/query/input/stream/state/receiver/ (all)
 * and emits one StateEvent per match into QuerySelector.process
 *   modules/siddhi-core/src/main/java/io/siddhi/core/query/selector/QuerySelector.java:76-99.
 * The entry points below replace, respectively:
 *   shp_engine_create   StateInputStreamParser.parseInputStream (:76-146) + QueryRuntimeImpl.start
 *   shp_push_batch      ProcessStreamReceiver.receive(long, Object[]) for a run of sends, including
 *                       PartitionStreamReceiver.send (core/partition/PartitionStreamReceiver.java:262-283)
 *                       and the playback clock (core/stream/input/InputHandler.java:59-70)
 *   shp_advance_clock   TimestampGeneratorImpl.setCurrentTimestamp (core/util/timestamp/
 *                       TimestampGeneratorImpl.java:105-121) with no event (timer flush)
 *   shp_snapshot/restore State.snapshot / State.restore of the query's state (SnapshotService)
 *   shp_engine_destroy  SiddhiAppRuntime.shutdown for the query
 * Errors are status codes (no exceptions cross the ABI); shp_last_error() gives text.
 * A single engine is not re-entrant (the reference serialises a query with
 * synchronized(patternSyncObject), SingleProcessStreamReceiver.java:52).
 */
#ifndef SIDDHI_HIP_H
#define SIDDHI_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SHP_OK 0
#define SHP_ERR_ARG -1          /* bad argument / malformed program JSON */
#define SHP_ERR_UNSUPPORTED -2  /* construct outside the state path */
#define SHP_ERR_CAPACITY -3     /* a per-key table overflowed (partials, chains, timers) */
#define SHP_ERR_OUTPUT -4       /* match buffer too small for this batch */
#define SHP_ERR_DEVICE -5       /* HIP runtime error */
#define SHP_ERR_KEYS -6         /* key id >= cfg.max_keys */

typedef struct shp_engine shp_engine;

typedef struct shp_config {
  int32_t device;          /* HIP device ordinal */
  int32_t max_keys;        /* partition-key dictionary capacity (1 when not partitioned) */
  int64_t max_batch;       /* largest n accepted by one push */
  int64_t max_matches;     /* match-record capacity per push */
  int64_t start_clock;     /* event-time clock at start() (0 in playback mode) */
  int32_t force_general;   /* 0 auto; 1 general NFA lanes only; 2 no sweep path (scan kernels or
                              lanes); 3 sweep path whenever the shape allows (any key count).
                              The count-sequence path (3) and the logical-absent path (4, the
                              playback pattern `every (x=X and y=Y) -> not Z for T [within W]`,
                              exact for any timestamp order; labs.h) are taken for their shapes
                              unless 1.  4: require the logical-absent path (create fails for
                              another shape). */
  int32_t profile_kernels; /* 1: time every kernel of a push with HIP events (shp_last_kernel_ms) */
  int32_t match_layout;    /* SHP_LAYOUT_FULL (0), SHP_LAYOUT_PAIRS (1), SHP_LAYOUT_AGG (2),
                              SHP_LAYOUT_PAIRS32 (3), SHP_LAYOUT_CHAIN32 (4) or SHP_LAYOUT_COMPACT (5);
                              PAIRS and PAIRS32 need the sweep path, CHAIN32 the count-sequence path */
} shp_config;

/* Match layouts. FULL: every field of shp_matches is valid. PAIRS (2-state sweep path,
 * device pushes): only `refs` is written, as m pairs (e1 seq, e2 seq); the other fields are
 * implied: ref_off[i] = 2i, slot_len = {1, 1}, pos = ts-event = refs[2i+1], type CURRENT,
 * key/ts = those of event refs[2i+1] in the pushed batch. shp_fetch_matches expands them. */
#define SHP_LAYOUT_FULL 0
#define SHP_LAYOUT_PAIRS 1
/* PAIRS32 (as PAIRS, half the bytes): `refs` holds m pairs of uint32 (e2's index in the pushed
 * batch, e2 seq - e1 seq): e2 seq = batch seq0 + index, e1 seq = e2 seq - delta.  A match whose
 * events are 2^32 or more events apart fails the push with SHP_ERR_UNSUPPORTED. */
#define SHP_LAYOUT_PAIRS32 3
/* AGG (sweep path, program with an "aggregate" select item): the selector's running aggregate
 * is computed on the device (replaces QuerySelector.processInBatchNoGroupBy with
 * AvgAttributeAggregatorExecutor / Sum / Count, core/query/selector/QuerySelector.java:271-313).
 * Only `key` and `agg` are written: match i is one output row (partition key, the aggregate's
 * value after that match, double), in per-key emission order. The aggregate state per key
 * carries across pushes. Null values in the aggregated column are rejected (SHP_ERR_UNSUPPORTED). */
#define SHP_LAYOUT_AGG 2
/* CHAIN32 (count-sequence path, `[every] e1=S[f1]<min:M>, e2=S[f2]` in a partition): `refs` holds m
 * uint32 words, word = e2's index in the pushed batch (bits 0-27) | L << 28.  The match's e1 chain
 * is the L events of e2's partition key immediately before e2 in that key's arrival order (the
 * pattern is a sequence: CountPreStateProcessor.java:53-95 keeps them consecutive), some possibly
 * from earlier pushes; the other fields are implied as for PAIRS (type CURRENT, ts / pos of e2,
 * slot_len {L, 1}).  shp_fetch_matches / shp_group_gather_matches expand to FULL.  Needs
 * max_batch < 2^28. */
#define SHP_LAYOUT_CHAIN32 4
/* COMPACT: the engine's own compact form, resolved at create -- PAIRS32 on the sweep path, CHAIN32 on
 * the count-sequence path, FULL on every other (shp_engine_stat(e, "match_layout") reports it).  For a
 * host that decodes every layout (the Java binding, with shp_push_batch_compact). */
#define SHP_LAYOUT_COMPACT 5

/* One batch of events in SoA form. Column c follows program["columns"][c]:
 * int->int32, long->int64, float->float32, double->float64, bool->uint8,
 * string->int32 (dictionary id, host owns the strings). nulls[c] may be NULL.
 * stream -1 marks a clock-only event: a send on a stream this query does not read, which in
 * playback still sets the app's clock (InputHandler.java:59-64) and so fires timers. */
typedef struct shp_batch {
  int64_t n;
  const int64_t* ts;
  const int32_t* key;      /* partition key id per event (0 when not partitioned) */
  const int32_t* stream;   /* stream index per event (program["streams"] order); NULL = all 0 */
  const void* const* cols;
  const uint8_t* const* nulls;
  /* optional (NULL = derived): the playback clock each event hands
   * TimestampGeneratorImpl.setCurrentTimestamp (core/util/timestamp/TimestampGeneratorImpl.java:
   * 105-121), the events' own ts when NULL.  A key-sharded rank sees only its keys' events, so it
   * is given the global clock here (AbsentStreamPreStateProcessor.java:216-223 reads it as
   * actualCurrentTime).  Used by the general NFA lanes (absent-state timers); the 2-state paths
   * have no timers and ignore it. */
  const int64_t* clock;
  /* optional: the events' sequence numbers (NULL = the engine's running count); match records
   * then refer to events by these numbers (a key-sharded rank passes global ones).  Not with
   * SHP_LAYOUT_PAIRS (its records must map back to batch positions). */
  const int64_t* seq;
} shp_batch;

/* Engine-owned match records (valid until the next call on the engine).
 * Per key, records are in reference emission order; across keys unspecified.
 * Slot s of match i holds slot_len[i*S+s] event sequence numbers starting at
 * refs[ref_off[i]] + sum_{t<s} slot_len[i*S+t]; seq -1 = an empty event. */
typedef struct shp_matches {
  int64_t m;
  int32_t num_states;      /* S */
  const int32_t* key;
  const int64_t* ts;       /* StateEvent timestamp (last matched event ts or timer due time) */
  const int8_t* type;      /* 0 CURRENT, 1 EXPIRED */
  const int64_t* pos;      /* event seq during (before, for timers) which the match was emitted */
  const int64_t* ref_off;
  const int16_t* slot_len;
  const int64_t* refs;
  int32_t layout;          /* SHP_LAYOUT_FULL, _PAIRS, _AGG, _PAIRS32 or _CHAIN32 */
  const double* agg;       /* SHP_LAYOUT_AGG: the aggregate's value per match */
} shp_matches;

int shp_engine_create(const char* nfa_program_json, const shp_config* cfg, shp_engine** out);

/* ---- SiddhiQL lowering inside the library (siddhi_amd/csrc/siddhiql.cpp) ----
 * The Java host keeps SiddhiQL (north_star); it hands the engine the app text and the query's name
 * instead of a pre-lowered program.  The lowering restates StateInputStreamParser.parse
 * (core/util/parser/StateInputStreamParser.java:148-408: state ids, next/every/partner wiring,
 * within, count min/max) and ExpressionParser.parseExpression / parseVariable
 * (ExpressionParser.java:223-557, 1253-1416: CURRENT / LAST index rules, Java numeric promotion)
 * for the state path's grammar (SiddhiQL.g4:200-345), and emits the program JSON byte-identical to
 * siddhi_amd/query/compiler.py.
 * String constants of the filters are interned in a shp_dict: the host encodes its string column
 * values with the same dictionary (shp_dict_intern), so constant and value ids agree.  A dict with
 * max_ids > 0 refuses new strings past that many (SHP_ERR_KEYS): a partition-key dictionary bounded
 * by cfg.max_keys (replaces the per-key state lookup of PartitionStateHolder.getState,
 * core/util/snapshot/state/PartitionStateHolder.java:43-48).  Dictionaries are thread-safe. */
typedef struct shp_dict shp_dict;
shp_dict* shp_dict_create(int32_t max_ids);
int32_t shp_dict_intern(shp_dict* d, const char* utf8, int64_t len);  /* id >= 0, or a status */
int32_t shp_dict_size(shp_dict* d);
int64_t shp_dict_string(shp_dict* d, int32_t id, char* out, size_t cap);
void shp_dict_destroy(shp_dict* d);
/* The program JSON of the app's query `query_name` (its @info(name=...), or "query<N>" by position;
 * NULL = the first query).  Writes at most cap bytes (NUL-terminated) and returns the full length,
 * or SHP_ERR_ARG (SiddhiParserException) / SHP_ERR_UNSUPPORTED (SiddhiAppCreationException:
 * a construct outside the state path); shp_compile_last_error() gives the text (per thread). */
int64_t shp_compile_siddhiql(const char* app_text, const char* query_name, shp_dict* dict, char* out, size_t cap);
/* The app's queries as JSON [{name, type, out, output_events, playback, partition: {stream: attr} |
 * null}], so the host can map its QueryRuntimes to names.  Same return convention. */
int64_t shp_siddhiql_queries(const char* app_text, char* out, size_t cap);
const char* shp_compile_last_error(void);
/* shp_compile_siddhiql + shp_engine_create in one call (the Java host's entry point). */
int shp_engine_create_siddhiql(const char* app_text, const char* query_name, shp_dict* dict, const shp_config* cfg,
                               shp_engine** out);

/* Host-memory batch: copied to HBM, processed, matches copied back to host memory. */
int shp_push_batch(shp_engine* e, const shp_batch* in, shp_matches* out);
/* HBM-resident batch (device pointers); matches stay in HBM (out holds device pointers).  With a
 * compact layout (PAIRS, PAIRS32, CHAIN32) the batch's device columns (ts, key, stream, seq) must stay
 * valid until the matches are fetched: shp_fetch_matches / shp_group_gather_matches expand the
 * compact records from them.  Key ids are the caller's here: keep them dense in [0, max_keys) (as
 * shp_dict issues them) -- the sweep spreads keys over its owners by the low bits of the id, so
 * strided ids run on a few owners (exact, but slow). */
int shp_push_batch_device(shp_engine* e, const shp_batch* in, shp_matches* out);
/* Host-memory batch with compact match records: as shp_push_batch, but the records come back in the
 * layout the engine produced them in, copied to host memory without expansion -- out->layout says
 * which: PAIRS32 / PAIRS (sweep path, `refs` holds the 32- / 64-bit words), CHAIN32 (count-sequence
 * path), AGG, or FULL on every other path.  Per key the compact records are in reference emission
 * order; across keys in owner order, so a host restoring the global order sorts them stably by
 * e2's batch index (the reference emits at e2's arrival, PatternSingleProcessStreamReceiver).
 * The Java binding's push (GpuStateStreamRuntime.flush). */
int shp_push_batch_compact(shp_engine* e, const shp_batch* in, shp_matches* out);
/* Pipelined host ingest: the host copy of batch i+1 overlaps the engine's run of
 * batch i.  shp_stage_batch enqueues the H2D copies of a host batch into one of two device slots on a
 * copy stream and returns at once (the host columns must stay valid and unchanged until the
 * shp_run_staged that consumes them returns; page-locked memory -- shp_host_alloc / shp_host_register
 * -- makes the copies asynchronous).  At most two batches are staged (a third: SHP_ERR_CAPACITY).
 * shp_run_staged runs the oldest staged batch as shp_push_batch_compact would (same state, same
 * records, in the engine's compact layout) and copies the records into page-locked memory owned by
 * the engine (valid until the next call).  Order: stage(0), stage(1), run -> 0, stage(2), run -> 1, ...
 * shp_stage_batch_ts32 is the narrow form: ts[i] = ts_base + ts_delta[i] (in->ts is ignored), 12
 * instead of 16 bytes per event for a float column -- the host keeps a batch's ts span below 2^31 ms. */
int shp_stage_batch(shp_engine* e, const shp_batch* in);
int shp_stage_batch_ts32(shp_engine* e, const shp_batch* in, int64_t ts_base, const int32_t* ts_delta);
/* The narrowest form: ts offsets as above and, with key16 != NULL, 2-byte partition key ids (in->key is
 * ignored; needs max_keys <= 65536, else SHP_ERR_ARG): 10 bytes per event for one float column. */
int shp_stage_batch_narrow(shp_engine* e, const shp_batch* in, int64_t ts_base, const int32_t* ts_delta,
                           const uint16_t* key16);
int shp_run_staged(shp_engine* e, shp_matches* out);
/* The oldest event sequence number the engine's committed state still names: an event of any open
 * partial (pending / new-and-every lists, count chains, logical slots, pairs waiting on an absent
 * timer, sweep carry).  Every later match names events >= this or of later pushes, so a host that
 * rebuilds StreamEvents from its own copy of the rows (ColumnarBatch) may drop the rows below it
 * -- the reference keeps a StreamEvent alive exactly as long as a partial holds it
 * (StreamPreStateProcessor.java:364-403).  The engine's next sequence number when nothing is open.
 * Costs a snapshot (device to host copy of the state): call it when the kept rows grow, not per push. */
int shp_engine_oldest_live_seq(shp_engine* e, int64_t* out);
/* The earliest due time among the keys' absent-state timers of the committed state: the head of each
 * key's Scheduler queue (a FIFO, core/util/Scheduler.java:113-127, 332).  Returns 1 and writes *out
 * when a timer is pending, 0 when none is (the 2-state and count-sequence paths have no timers), or a
 * negative status.  A live-mode (non-playback) host schedules a wall-clock wake-up at that time and
 * then calls shp_advance_clock(now), as Scheduler.schedule / EventCaller.run do (:129-155, :287-326).
 * Costs a snapshot (device to host copy of the state), as shp_engine_oldest_live_seq. */
int shp_engine_next_due(shp_engine* e, int64_t* out);
/* Copy the matches of the last shp_push_batch_device to host memory (none after shp_restore). */
int shp_fetch_matches(shp_engine* e, shp_matches* out);
int shp_advance_clock(shp_engine* e, int64_t now, shp_matches* out);
/* Per-key state of the engine (partial matches, carried candidates, timers, clock, sequence
 * numbers) as an opaque blob (engine-owned, valid until the next snapshot or destroy), and its
 * restore into an engine created from the same program with the same path and max_keys.
 * Replaces State.snapshot()/restore() (core/util/snapshot/state/State.java:25-36) as driven by
 * SnapshotService (core/util/snapshot/SnapshotService.java:90-188) for the query. */
int shp_snapshot(shp_engine* e, void** buf, size_t* len);
int shp_restore(shp_engine* e, const void* buf, size_t len);
/* A snapshot of this engine decoded into the reference's State.snapshot() key names, as JSON:
 * {"engine": {path, seq, clock}, "keys": {"<key id>": {"<state>": {"FirstEvent",
 * "PendingStateEventList", "NewAndEveryStateEventList", "Initialized", "Started"
 * (StreamPreStateProcessor.java:450-469), count states also "SuccessCondition", "StartStateReset"
 * (CountPreStateProcessor.java:206-219), absent states "IsActive", "LastScheduledTime",
 * "LastArrivalTime" (AbsentStreamPreStateProcessor.java:328-341)}, "scheduler<i>": {"ToNotifyQueue"}
 * (Scheduler.java:349-360)}}}; a partial is {ts, type, slots: per state the [{seq, ts}] chain}.
 * Writes at most cap bytes (NUL-terminated) and returns the full length, or a negative status. */
int64_t shp_snapshot_describe(shp_engine* e, const void* buf, size_t len, char* out, size_t cap);
int shp_engine_num_states(const shp_engine* e);
/* The stream (index in the program's "streams" order, i.e. the receiver) state `state` reads, or
 * -1.  States are numbered as StateInputStreamParser.parse adds their MetaStreamEvents
 * (core/util/parser/StateInputStreamParser.java:167-177: stateIndex = getStreamEventCount() - 1),
 * so a host builds one SingleStreamRuntime per state, in MetaStateEvent order, on the receiver of
 * this stream (QueryParserHelper.initStreamRuntime indexes getSingleStreamRuntimes() by state,
 * core/util/parser/helper/QueryParserHelper.java:161-167). */
int shp_engine_state_stream(const shp_engine* e, int state);
/* Which kernels the engine runs: 2 = sweep (owner partition + LDS sweep), 1 = specialised 2-state
 * scan kernel, 0 = general NFA lanes, 3 = count-sequence automaton (`[every] e1=S[f1]<min:M>,
 * e2=S[f2]` with f2 over e2 and e1[last], 1 <= min <= M <= 8, no within; siddhi_amd/csrc/cseq.h),
 * 4 = logical-absent (`every (x and y) -> not z for T` in playback: the default for that shape,
 * exact for any timestamp order; siddhi_amd/csrc/labs.h).  A path-3 snapshot
 * describes each key as {"e1": {"Count": L, "PendingStateEventList": [the chain partial]},
 * "LastEvent": {seq, ts}}. */
int shp_engine_path(const shp_engine* e);
/* ---- Key-sharded multi-GPU (SURVEY.md §8b "Multi-GPU is internal to the engine", §8e) ----
 * A partitioned query's keys are split over `world` engines: key k on rank k % world (the dense
 * id k / world there).  One push hands every rank one slice of the global stream (consecutive
 * pieces in rank order, device pointers on that rank's GPU); the group splits each slice by key
 * owner on the GPU, exchanges it (RCCL ncclSend/ncclRecv over xGMI between processes, device
 * copies within one process), and every rank's engine runs the keys it owns.  Per-key emission
 * order is the reference's (a key lives on one rank; received events keep global order).  The
 * group's cfg.max_keys is the global key count; cfg.max_batch bounds the events one rank may
 * receive per push.  Absent-state timers get the global playback clock (shp_batch.clock), so a
 * timer match carries the reference's ts (the due time) and slots; its `pos` (the sequence number
 * of the event during which it was emitted) is the owning rank's next event, not necessarily the
 * global next event -- the one documented divergence of a sharded run from one engine (per-key
 * record order and every other field are the reference's);
 * SHP_LAYOUT_FULL records name events by global sequence number.  Replaces, for the sharded
 * deployment, PartitionStreamReceiver.receive/send (core/partition/PartitionStreamReceiver.java:
 * 82-283) routing each event to its key's state. */
typedef struct shp_group shp_group;
#define SHP_COMM_ID_BYTES 128
/* One process driving `world` GPUs (e.g. one JVM): rank r on devices[r] (repeats allowed). */
int shp_group_create(const char* nfa_program_json, const shp_config* cfg, int32_t world, const int32_t* devices,
                     shp_group** out);
/* One process per GPU: rank 0 makes the RCCL id, the host broadcasts its SHP_COMM_ID_BYTES bytes,
 * every rank then creates its member on cfg.device (a collective call). */
int shp_comm_id(void* id, size_t len);
int shp_group_create_rank(const char* nfa_program_json, const shp_config* cfg, int32_t world, int32_t rank,
                          const void* comm_id, shp_group** out);
/* One push (collective: every rank pushes once per step).  slices: one shp_batch per local rank
 * (in-process group: world of them; per-rank member: its own).  matches (may be NULL): per local
 * rank, the matches of this push (they stay in HBM until shp_group_fetch_matches). */
int shp_group_push(shp_group* g, const shp_batch* slices, int64_t* matches);
/* shp_group_push in two halves, so the exchange of later batches overlaps the engines' run of
 * this one: stage = split + exchange into one of three receive slots (returns once the exchange
 * is enqueued; the slices must stay valid until that batch's run returns); run = the engines on
 * the oldest staged batch.  At most three batches staged ahead; one thread may stage while
 * another runs (and nothing else calls into the group meanwhile). */
int shp_group_stage(shp_group* g, const shp_batch* slices);
int shp_group_run(shp_group* g, int64_t* matches);
/* The local ranks' matches of the last push in host memory, global key ids, per-key emission order. */
int shp_group_fetch_matches(shp_group* g, shp_matches* out);
/* Every rank's matches of the last push gathered to rank `root` (a collective call: every rank of
 * a one-process-per-GPU group calls it).  The records move in HBM (RCCL send / recv to the root,
 * or device copies within one process); global key ids, ranks in order, per-key emission order.
 * The root's out holds host pointers (valid until the next gather); other ranks get m = 0.
 * "the matches are ncclGather'ed to rank 0". */
int shp_group_gather_matches(shp_group* g, int32_t root, shp_matches* out);
int shp_group_local_engines(const shp_group* g);
shp_engine* shp_group_engine(shp_group* g, int32_t i);  /* local rank i's engine (timings, snapshots) */
const char* shp_group_last_error(const shp_group* g);
void shp_group_destroy(shp_group* g);

/* Bench/test utility (not part of the reference boundary): fill device buffers with events
 * start..start+count-1 of the SURVEY.md §8d synthetic stream (PCG32, bit-identical to
 * siddhi_amd/synth.py). Any output pointer may be NULL. hip_stream: a hipStream_t or NULL. */
int shp_synth_fill(int config, int64_t start, int64_t count, int64_t keys, int n_streams, int dense,
                   int64_t* ts, int32_t* key, float* price, int64_t* volume, int32_t* stream, void* hip_stream);
/* Multi-GPU exchange utilities (not part of the reference boundary; siddhi_amd/shard.py):
 * stable split of a device batch by destination rank key % G into packed 16-byte records
 * {ts, stream << 24 | key / G, value} grouped by rank (counts[g] on the host), and the unpack of
 * received records into the engine's SoA columns. */
int64_t shp_shard_workspace_bytes(int64_t n, int G);
int shp_shard_partition(int64_t n, const int64_t* ts, const int32_t* key, const void* value, const int32_t* stream,
                        int G, void* out, int64_t* counts, void* ws, void* hip_stream);
int shp_shard_unpack(int64_t m, const void* in, int64_t* ts, int32_t* key, void* value, int32_t* stream,
                     void* hip_stream);
/* The same split into destination-grouped SoA columns (out_key = key / G; out_value / out_stream
 * NULL when value / stream is): one all-to-all per column lands the owner's engine input as is. */
int shp_shard_partition_soa(int64_t n, const int64_t* ts, const int32_t* key, const void* value,
                            const int32_t* stream, int G, int64_t* out_ts, int32_t* out_key, void* out_value,
                            int32_t* out_stream, int64_t* counts, void* ws, void* hip_stream);
/* Bench/test utilities: device memory without a second HIP runtime in the process. */
void* shp_dev_alloc(int64_t bytes);
int shp_dev_free(void* p);
int shp_dev_to_host(void* dst, const void* src, int64_t bytes);
/* Page-locked host memory for match payloads (hipHostMalloc / hipHostRegister): a D2H copy into it
 * runs at DMA rate.  A Java host pins its receive MemorySegment once with shp_host_register. */
void* shp_host_alloc(int64_t bytes);
int shp_host_free(void* p);
int shp_host_register(void* p, int64_t bytes);
int shp_host_unregister(void* p);
/* Device time (ms) of the last push measured with HIP events on the engine stream:
 * which = "total" | "partition" | "nfa" | a kernel name (needs cfg.profile_kernels), e.g.
 * "radix_sort", "nfa_lanes", "fast_search", "fast_emit". */
double shp_last_kernel_ms(const shp_engine* e, const char* which);
/* Engine counters since create: which = "pushes" | "lean_pushes" (sweep pushes run by the
 * k_sw_lean solve) | "lean_fallbacks" (of those, pushes that
 * k_sw_lean handed back to the exact k_sw_solve: a ts decrease within a key, a push spanning
 * more than 2^30 ms, a large carry) | "labs_fallbacks" (logical-absent pushes that k_labs_w, a
 * wave per key, handed to k_labs, a thread per key: a key with more than 64 pairs waiting at
 * once) | "cseq_wide_reruns" (count-sequence pushes whose ts span more than +-2^31 ms of their
 * first ts, re-run with 16-byte records) | "spill_reruns" | "spilled_owners".  -1 for an unknown
 * name. */
int64_t shp_engine_stat(const shp_engine* e, const char* which);
const char* shp_last_error(const shp_engine* e);
void shp_engine_destroy(shp_engine* e);

#ifdef __cplusplus
}
#endif
#endif /* SIDDHI_HIP_H */
