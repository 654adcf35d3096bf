"""CPU checks of the Java (Panama FFM) binding under java/ -- there is no JDK in this image, so the
sources are checked as text against the C header compiled with gcc and against the program the
library lowers:

* ShpNative.java's struct layouts (CONFIG, BATCH, MATCHES: field list, padding, size) and the CFG_*
  offsets GpuStateStreamRuntime fills shp_config by, against offsetof/sizeof of include/siddhi_hip.h;
* every symbol a downcall handle names is declared in the header, and every ShpNative handle the
  other Java files use exists;
* GpuStateStreamRuntime returns one SingleStreamRuntime per state (the reference's query builder
  indexes getSingleStreamRuntimes() by state, QueryParserHelper.java:161-167), built from
  shp_engine_state_stream;
* the state numbering of every lowered fixture app is the reference's MetaStateEvent order: the
  order StateInputStreamParser.parse reaches the stream states (Next: current then next,
  StateInputStreamParser.java:227-262; Logical: the second operand first, :336-351; Every and
  Count: their inner state), and each state's stream is the one it reads -- the map the Java side
  pairs receivers and MetaStreamEvents by (ProgramInfo.stateStream, shp_engine_state_stream).
"""
import json
import os
import re
import subprocess
import tempfile

import pytest

from golden_runner import load_fixtures
from siddhi_amd import native, synth
from siddhi_amd.query.compiler import Dictionary, QueryCompiler
from siddhi_amd.query.siddhiql import parse_app

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JAVA = os.path.join(ROOT, "java", "io", "siddhi", "core", "query", "input", "stream", "state", "gpu")
SIZES = {"JAVA_INT": (4, 4), "JAVA_LONG": (8, 8), "ADDRESS": (8, 8), "JAVA_DOUBLE": (8, 8), "JAVA_SHORT": (2, 2),
         "JAVA_BYTE": (1, 1)}


def _java(name):
    return open(os.path.join(JAVA, name)).read()


def _struct_layouts(src):
    """{LAYOUT: [(field or None for padding, offset, size)], total size} from ShpNative's
    MemoryLayout.structLayout(...) declarations (natural alignment, as the FFM linker requires)."""
    out = {}
    for name, body in re.findall(r"static final StructLayout (\w+) = MemoryLayout\.structLayout\((.*?)\);", src, re.S):
        fields, off, align = [], 0, 1
        for m in re.finditer(r"(JAVA_\w+|ADDRESS)\.withName\(\"(\w+)\"\)|MemoryLayout\.paddingLayout\((\d+)\)", body):
            if m.group(3):
                n = int(m.group(3))
                fields.append((None, off, n))
                off += n
                continue
            sz, al = SIZES[m.group(1)]
            assert off % al == 0, f"{name}.{m.group(2)} misaligned at {off}"
            fields.append((m.group(2), off, sz))
            off += sz
            align = max(align, al)
        assert off % align == 0, f"{name}: size {off} not a multiple of {align}"
        out[name] = (fields, off)
    return out


def _c_offsets(structs):
    """offsetof/sizeof of the header's structs, compiled with gcc."""
    body = []
    for st, fs in structs.items():
        body.append(f'printf("{st} %zu", sizeof({st}));')
        for f in fs:
            body.append(f'printf(" {f}=%zu", offsetof({st}, {f}));')
        body.append('printf("\\n");')
    src = ("#include <stdio.h>\n#include <stddef.h>\n#include \"siddhi_hip.h\"\nint main(void){" + "".join(body)
           + "return 0;}")
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "l.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "l")
        subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), "-o", exe, c])
        lines = subprocess.check_output([exe]).decode().strip().split("\n")
    res = {}
    for line in lines:
        parts = line.split()
        res[parts[0]] = (int(parts[1]), {k: int(v) for k, v in (p.split("=") for p in parts[2:])})
    return res


LAYOUT_STRUCT = {"CONFIG": "shp_config", "BATCH": "shp_batch", "MATCHES": "shp_matches"}


def test_shpnative_struct_layouts_match_the_header():
    lay = _struct_layouts(_java("ShpNative.java"))
    assert set(LAYOUT_STRUCT) <= set(lay)
    want = _c_offsets({LAYOUT_STRUCT[k]: [f for f, _, _ in lay[k][0] if f] for k in LAYOUT_STRUCT})
    for jname, cname in LAYOUT_STRUCT.items():
        fields, size = lay[jname]
        csize, coff = want[cname]
        assert size == csize, (jname, size, csize)
        named = [(f, o) for f, o, _ in fields if f]
        assert [f for f, _ in named] == list(coff), (jname, [f for f, _ in named], list(coff))
        for f, o in named:
            assert o == coff[f], f"{jname}.{f}: Java offset {o}, C offsetof {coff[f]}"
    # the sizes the Javadoc comments state
    src = _java("ShpNative.java")
    for jname, cname in LAYOUT_STRUCT.items():
        m = re.search(r"/\*\* struct " + cname + r" \((\d+) bytes\)", src)
        assert m and int(m.group(1)) == want[cname][0], cname


def test_config_is_filled_by_header_offsets():
    src = _java("ShpNative.java")
    consts = {k: int(v) for k, v in re.findall(r"CFG_(\w+) = (\d+)", src)}
    want = _c_offsets({"shp_config": [k.lower() for k in consts]})["shp_config"][1]
    assert consts and {k.lower(): v for k, v in consts.items()} == want
    rt = _java("GpuStateStreamRuntime.java")
    sets = re.findall(r"cfg\.set\((JAVA_\w+), ([^,]+),", rt)
    assert len(sets) == 8
    for typ, off in sets:  # every field written by its named offset, never a literal
        assert off.startswith("ShpNative.CFG_"), off
        field = off[len("ShpNative.CFG_"):].lower()
        assert field in want
        assert SIZES[typ][0] == (8 if field in ("max_batch", "max_matches", "start_clock") else 4), (typ, field)


def test_downcalls_name_declared_symbols():
    from test_abi import declared_symbols
    src = _java("ShpNative.java")
    named = set(re.findall(r"fn(?:Void)?\(\"(shp_\w+)\"", src))
    assert named, "no downcalls found"
    missing = named - set(declared_symbols())
    assert not missing, missing
    handles = set(re.findall(r"static final MethodHandle (\w+) =", src))
    for f in os.listdir(JAVA):
        if f.endswith(".java") and f != "ShpNative.java":
            used = set(re.findall(r"ShpNative\.([A-Z][A-Z0-9_]+)\.invokeExact", _java(f)))
            assert used <= handles, (f, used - handles)


def test_runtime_builds_one_single_stream_runtime_per_state():
    rt = _java("GpuStateStreamRuntime.java")
    body = rt[rt.index("GpuStateStreamRuntime(String appText, String queryName, ProgramInfo info"):]
    loop = re.search(r"for \(int st = 0; st < numStates; st\+\+\) \{(.*?)\n            \}", body, re.S)
    assert loop, "no per-state loop in the constructor"
    text = loop.group(1)
    assert "ShpNative.STATE_STREAM.invokeExact(eng, st)" in text
    assert "singleStreamRuntimes.add(new SingleStreamRuntime(receivers[s]" in text
    assert "metaStateEvent.getMetaStreamEvent(st)" in text
    # one receiver per stream, shared by the states that read it
    assert "if (receivers[s] == null)" in text
    assert rt.count("singleStreamRuntimes.add(") == 1


def _reference_state_order(tree):
    """State ids in the order StateInputStreamParser.parse adds their MetaStreamEvents."""
    t = tree["t"]
    if t in ("stream", "absent", "count"):
        return [tree["state"]]
    if t == "next":
        return _reference_state_order(tree["a"]) + _reference_state_order(tree["b"])
    if t == "every":
        return _reference_state_order(tree["x"])
    if t == "logical":  # getStreamStateElement2 is parsed before getStreamStateElement1
        return _reference_state_order(tree["s2"]) + _reference_state_order(tree["s1"])
    raise AssertionError(f"unknown tree node {t}")


def _reader(p, node_state_streams):
    """ProgramInfo.parse's per-state map, restated: state id -> stream, ref, count state."""
    st = {s["id"]: (s["stream"], s["ref"]) for s in p["states"]}
    multi = set()

    def walk(n):
        if isinstance(n, dict):
            if n.get("t") == "count":
                multi.add(n["state"])
            for v in n.values():
                walk(v)
    walk(p["tree"])
    return [(st[i][0], st[i][1], i in multi) for i in range(len(st))]


def _programs():
    seen = set()
    apps = [fx["app"] for fx in load_fixtures()] + list(synth.QUERIES.values())
    for app_text in apps:
        if app_text in seen:
            continue
        seen.add(app_text)
        try:
            app = parse_app(app_text)
        except Exception:  # noqa: BLE001 (apps outside the state path's grammar)
            continue
        d = Dictionary()
        for q in app.queries:
            try:
                yield app, q, json.loads(QueryCompiler(app, q, d).compile().program_json())
            except Exception:  # noqa: BLE001 (queries the lowering rejects: the host keeps the reference)
                break


def test_state_numbering_is_the_reference_meta_order():
    n = 0
    for app, q, p in _programs():
        order = _reference_state_order(p["tree"])
        assert order == list(range(len(p["states"]))), (q.name, order)
        streams = [s["name"] for s in p["streams"]]
        for sid, (stream, ref, multi) in enumerate(_reader(p, None)):
            assert 0 <= stream < len(streams)
        n += 1
    assert n >= 200


def test_state_stream_map_for_c2_and_c4():
    """C2: two states on one stream (two SingleStreamRuntimes, one receiver); C4: the logical
    element's second operand is state 0 (S2), so state order differs from stream order."""
    progs = {}
    for key in (2, 4):
        _, qs, _ = __import__("siddhi_amd.query.compiler", fromlist=["compile_app"]).compile_app(synth.QUERIES[key])
        progs[key] = json.loads(qs[0].program_json())
    assert [s for s, _, _ in _reader(progs[2], None)] == [0, 0]
    assert [s for s, _, _ in _reader(progs[4], None)] == [1, 0, 2]
    assert [r for _, r, _ in _reader(progs[4], None)] == ["e2", "e1", None]


@pytest.mark.gpu
def test_engine_state_stream_matches_the_program():
    """shp_engine_state_stream (what GpuStateStreamRuntime calls) on every lowered fixture query."""
    checked = 0
    for app, q, p in _programs():
        try:
            eng = native.HipEngine(json.dumps(p), 0, max_keys=64, max_batch=256)
        except native.ShpError:
            continue
        try:
            assert eng.state_streams == [s for s, _, _ in _reader(p, None)], q.name
            checked += 1
        finally:
            eng.close()
    assert checked >= 150


def test_layout_constants_match_the_header():
    """SHP_LAYOUT_* of include/siddhi_hip.h, ShpNative.LAYOUT_* and siddhi_amd.native.LAYOUT_* agree."""
    hdr = open(os.path.join(ROOT, "include", "siddhi_hip.h")).read()
    want = {k: int(v) for k, v in re.findall(r"#define SHP_LAYOUT_(\w+) (\d+)", hdr)}
    assert set(want) == {"FULL", "PAIRS", "AGG", "PAIRS32", "CHAIN32", "COMPACT"}
    java = {k: int(v) for k, v in re.findall(r"static final int LAYOUT_(\w+) = (\d+);", _java("ShpNative.java"))}
    assert java == want
    assert {k: getattr(native, "LAYOUT_" + k) for k in want} == want


# ------------------------------------------------------------------ partition wiring (8f-2)
REF_CORE = "/root/reference/modules/siddhi-core/src/main/java/io/siddhi/core"
# the supertypes the reference declares for the stream runtimes PartitionRuntimeImpl dispatches on
REF_SUPERS = {"StateStreamRuntime": ["StreamRuntime"], "SingleStreamRuntime": ["StreamRuntime"],
              "JoinStreamRuntime": ["StreamRuntime"]}


def _type_chain(src, cls):
    m = re.search(r"public (?:final )?class " + cls + r" (?:extends (\w+))?\s*(?:implements ([\w, ]+))?\{", src)
    assert m, f"no class declaration for {cls}"
    chain, todo = [cls], [t.strip() for t in (m.group(1) or "").split(",") + (m.group(2) or "").split(",") if t.strip()]
    while todo:
        t = todo.pop(0)
        chain.append(t)
        todo += REF_SUPERS.get(t, [])
    return chain


def _partition_branch(chain):
    """PartitionRuntimeImpl.addPartitionReceiver (core/partition/PartitionRuntimeImpl.java:243-258):
    the instanceof dispatch that decides whether a query's outer streams get PartitionStreamReceivers."""
    for t, branch in (("SingleStreamRuntime", "single"), ("JoinStreamRuntime", "join"), ("StateStreamRuntime", "state")):
        if t in chain:
            return branch
    return None  # no receiver: the query would never see a partitioned stream's events


def _wired_streams(tree, states, streams):
    """addPartitionReceiverForStateElement (:262-288): Every -> inner, Next -> current then next,
    Count -> inner, Logical -> element 1 then 2, stream -> one receiver with the next executor index."""
    out = []

    def walk(n):
        t = n["t"]
        if t == "every":
            walk(n["x"])
        elif t == "next":
            walk(n["a"])
            walk(n["b"])
        elif t == "logical":
            walk(n["s1"])
            walk(n["s2"])
        else:  # stream, count, absent: one StreamStateElement
            out.append(streams[states[n["state"]]["stream"]]["name"])
    walk(tree)
    return out


@pytest.mark.parametrize("cfg", [2, 3, "3b", 4, 5])
def test_partitioned_queries_reach_the_state_branch_and_subscribe_every_stream(cfg):
    """C2-C5 are partitioned: the runtime's type takes PartitionRuntimeImpl's StateStreamRuntime
    branch, every stream the query reads gets its PartitionStreamReceiver, and
    PartitionStreamReceiver.addStreamJunction (:291-310: for i < getInputStreamId().size(), subscribe
    runtime i's receiver when its stream is the junction's) subscribes one of our runtimes to each."""
    rt = _java("GpuStateStreamRuntime.java")
    chain = _type_chain(rt, "GpuStateStreamRuntime")
    assert _partition_branch(chain) == "state", chain
    app, qs, _ = parse_app_and_compile(cfg)
    prog = qs[0].program
    assert prog["partitioned"]
    wired = _wired_streams(prog["tree"], prog["states"], prog["streams"])
    read = {prog["streams"][s["stream"]]["name"] for s in prog["states"]}
    assert set(wired) == read and len(wired) == len(prog["states"])
    # getInputStreamId() = StateInputStream.getAllStreamIds (collectStreamIds: the same walk), and the
    # runtimes are ProgramInfo.stateStream in state order (one SingleStreamRuntime per state)
    runtime_stream = [prog["streams"][s["stream"]]["name"] for s in sorted(prog["states"], key=lambda s: s["id"])]
    for stream in set(wired):
        assert any(runtime_stream[i] == stream for i in range(len(wired))), (stream, runtime_stream)


def parse_app_and_compile(cfg):
    from siddhi_amd.query.compiler import compile_app
    return compile_app(synth.QUERIES[cfg])


def test_runtime_extends_state_stream_runtime_and_overrides_its_inner_runtime_calls():
    rt = _java("GpuStateStreamRuntime.java")
    assert "import io.siddhi.core.query.input.stream.state.StateStreamRuntime;" in rt
    ctor = rt[rt.index("GpuStateStreamRuntime(String appText, String queryName, ProgramInfo info"):]
    body = ctor[ctor.index("{") + 1:]
    # StateStreamRuntime(SiddhiQueryContext, MetaStateEvent) (StateStreamRuntime.java:44): first statement
    assert body.lstrip().startswith("super(queryContext, metaStateEvent);")
    # every StateStreamRuntime method that reads its innerStateRuntime (null here) is overridden
    for m in ("getSingleStreamRuntimes()", "setCommonProcessor(Processor", "resetAndUpdate()", "initPartition()",
              "getMetaComplexEvent()", "getProcessingMode()", "getQuerySelector()"):
        assert re.search(r"@Override\s+public [\w<>]+ " + re.escape(m), rt), m


@pytest.mark.skipif(not os.path.isdir(REF_CORE), reason="reference sources not present")
def test_reference_dispatch_is_the_one_restated():
    """The restated dispatch and walk are the reference's (read as text where the sources exist)."""
    src = open(os.path.join(REF_CORE, "partition", "PartitionRuntimeImpl.java")).read()
    assert "instanceof SingleStreamRuntime" in src and "instanceof JoinStreamRuntime" in src
    assert "} else if (queryRuntime.getStreamRuntime() instanceof StateStreamRuntime) {" in src
    st = open(os.path.join(REF_CORE, "query", "input", "stream", "state", "StateStreamRuntime.java")).read()
    assert "public class StateStreamRuntime implements StreamRuntime" in st
    for m in ("public void resetAndUpdate()", "public void initPartition()",
              "public StateStreamRuntime(SiddhiQueryContext siddhiQueryContext, MetaStateEvent metaStateEvent)"):
        assert m in st, m


def test_runtime_pushes_compact_and_trims_by_oldest_live_seq():
    """The Java flush follows the mirror's rules (siddhi_amd/runtime.py, tests/test_retention.py):
    SHP_LAYOUT_COMPACT, shp_push_batch_compact, commit then decode, trim by the engine's report;
    no fixed push-count history is left."""
    rt = _java("GpuStateStreamRuntime.java")
    cb = _java("ColumnarBatch.java")
    assert "ShpNative.CFG_MATCH_LAYOUT, ShpNative.LAYOUT_COMPACT" in rt
    assert "ShpNative.PUSH_BATCH_COMPACT.invokeExact(engine, batch.descriptor(), matches)" in rt
    flush = rt[rt.index("void flush()"):rt.index("private long oldestLiveSeq()")]
    assert flush.index("batch.commit()") < flush.index("deliver(seq0, pushed)") < flush.index("batch.maybeTrim(")
    assert "ShpNative.OLDEST_LIVE_SEQ.invokeExact(engine, out)" in rt
    for dec in ("deliverPairs32", "deliverChain32", "deliverFull"):
        assert f"private void {dec}(" in rt
    assert "historyBatches" not in cb and "history.size() >" not in cb
    assert "void maybeTrim(LongSupplier oldestLive)" in cb and "void trim(long lo)" in cb
    src = _java("ShpNative.java")
    assert re.search(r"LAYOUT_COMPACT = 5;", src)


def _method(src, sig):
    """The body of the method whose declaration contains `sig` (brace-matched)."""
    i = src.index(sig)
    j = src.index("{", i)
    depth = 0
    for k in range(j, len(src)):
        depth += {"{": 1, "}": -1}.get(src[k], 0)
        if depth == 0:
            return src[j:k + 1]
    raise AssertionError(sig)


def test_every_match_reaches_the_selector_inside_its_partition_flow():
    """Egress as the reference: PartitionStreamReceiver.send (:262-272) and the Scheduler's timer loop
    (Scheduler.java:88-97) run a match under SiddhiAppContext.startPartitionFlow(key), and the selector's
    per-key state is looked up under it (PartitionStateHolder.java:43-48).  selector.process appears only
    inside emit(), which sets the match key's flow and restores the caller's in a finally; each decoder
    hands emit the key of its record (PAIRS32 / CHAIN32: the batch's key column, FULL: the records')."""
    rt = _java("GpuStateStreamRuntime.java")
    code = re.sub(r"/\*.*?\*/|//[^\n]*", "", rt, flags=re.S)
    emit = _method(code, "private void emit(int keyId, StateEvent se)")
    assert code.count("selector.process(") == emit.count("selector.process(") == 2
    assert "SiddhiAppContext.startPartitionFlow(keys.string(keyId))" in emit
    fin = emit[emit.index("finally"):]
    assert "SiddhiAppContext.startPartitionFlow(prev)" in fin and "SiddhiAppContext.stopPartitionFlow()" in fin
    assert emit.index("SiddhiAppContext.getPartitionFlowId()") < emit.index("startPartitionFlow(keys.string")
    assert "emit(batch.keyAt(idx), se)" in _method(code, "private void deliverPairs32(")
    assert "emit(k, se)" in _method(code, "private void deliverChain32(")
    full = _method(code, "private void deliverFull(")
    assert 'matchesPtr(matches, "key", m * 4)' in full and "emit(key.getAtIndex(JAVA_INT, i), se)" in full
    nd = _java("NativeDictionary.java")
    assert "String string(int id)" in nd and "ShpNative.DICT_STRING.invokeExact" in nd


def test_the_app_clock_reaches_the_engine():
    """Clock as the reference's Scheduler hears it: a TimeChangeListener on the app's TimestampGenerator
    (Scheduler.java:71-72) for queries with an absent state -- SYNC advances the engine at once, DEFERRED
    appends a clock-only row that the following event of the same send absorbs; live mode keeps one
    wall-clock wake-up at shp_engine_next_due (Scheduler.java:129-155) that advances to the wall clock."""
    rt = re.sub(r"/\*.*?\*/|//[^\n]*", "", _java("GpuStateStreamRuntime.java"), flags=re.S)
    assert "getTimestampGenerator().addTimeChangeListener(this::onTimeChange)" in rt
    ctor = rt[rt.index("GpuStateStreamRuntime(String appText"):rt.index("private void rethrowDeferred()")]
    assert "if (timers)" in ctor and "addTimeChangeListener" in ctor
    otc = _method(rt, "void onTimeChange(long now)")
    assert "advanceClock(now)" in otc and "batch.appendClock(now)" in otc
    assert otc.index("FlushPolicy.SYNC") < otc.index("advanceClock(now)") < otc.index("batch.appendClock(now)")
    wake = _method(rt, "private void scheduleWake()")
    assert "appContext.isPlayback()" in wake and "nextDue()" in wake
    assert "getScheduledExecutorService().schedule(this::onWake" in wake
    assert "ShpNative.NEXT_DUE.invokeExact(engine, out)" in _method(rt, "private long nextDue()")
    assert "advanceClock(appContext.getTimestampGenerator().currentTime())" in _method(rt, "private void onWake()")
    for m in ("void flush()", "void advanceClock(long now)"):
        assert "scheduleWake();" in _method(rt, m), m
    pi = _java("ProgramInfo.java")
    assert 'timers |= Boolean.TRUE.equals(m.get("absent"))' in pi
    cb = re.sub(r"/\*.*?\*/|//[^\n]*", "", _java("ColumnarBatch.java"), flags=re.S)
    app = _method(cb, "void append(long timestamp, int keyId, int streamIndex, Object[] data)")
    assert ("streamIndex >= 0 && n > 0 && o.stream.getAtIndex(JAVA_INT, n - 1) < 0" in app
            and "o.rowTs.get((int) n - 1) == timestamp" in app)
    assert "append(now, 0, -1, null)" in _method(cb, "void appendClock(long now)")


def test_columnar_batch_finds_rows_by_bisection_and_restore_validates():
    """event() bisects the kept blocks by seq0 (history is unbounded, trimmed only to the
    engine's oldest live seq); restoreFrom refuses a snapshot without the rows before touching the engine."""
    cb = re.sub(r"/\*.*?\*/|//[^\n]*", "", _java("ColumnarBatch.java"), flags=re.S)
    ev = _method(cb, "StreamEvent event(long seq, int outputDataSize)")
    assert "(lo + hi) >>> 1" in ev and "descendingIterator" not in ev
    rt = re.sub(r"/\*.*?\*/|//[^\n]*", "", _java("GpuStateStreamRuntime.java"), flags=re.S)
    rf = _method(rt, "void restoreFrom(Map<String, Object> m)")
    assert rf.index('m.get("LiveRows") instanceof Object[]') < rf.index("restore((byte[])")


def test_pipelined_flush_stages_then_runs_the_older_batch():
    """FlushPolicy.PIPELINED (the mirror: SiddhiAppRuntime(pipelined=True), tests/test_flow_clock.py):
    flush stages the open rows (shp_stage_batch from page-locked column sets) and runs the batch staged
    before them (shp_run_staged), committing its rows in run order; every point that observes state
    (advanceClock, snapshot, restore, shutdown) drains the staged batches first."""
    rt = re.sub(r"/\*.*?\*/|//[^\n]*", "", _java("GpuStateStreamRuntime.java"), flags=re.S)
    assert "enum FlushPolicy { SYNC, DEFERRED, PIPELINED }" in rt
    fl = _method(rt, "void flush()")
    assert fl.index("stageOpen()") < fl.index("runStaged()") < fl.index("PUSH_BATCH_COMPACT")
    assert "batch.stagedCount() > (fresh ? 1 : 0)" in fl
    st = _method(rt, "private boolean stageOpen()")
    assert "ShpNative.STAGE_BATCH.invokeExact(engine, batch.descriptor())" in st
    assert st.index("invokeExact") < st.index("batch.markStaged()")
    run = _method(rt, "private void runStaged()")
    assert run.index("batch.stagedSize()") < run.index("ShpNative.RUN_STAGED.invokeExact(engine, matches)")
    assert run.index("RUN_STAGED") < run.index("batch.commitStaged()") < run.index("deliver(seq0, pushed)")
    assert run.count("batch.dropStaged()") == 2
    dr = _method(rt, "private void drain()")
    assert "while (batch.stagedCount() > 0)" in dr
    for m in ("void advanceClock(long now)", "byte[] snapshot()", "public void shutdown()"):
        assert "drain();" in _method(rt, m), m
    assert "runStaged()" in _method(rt, "void restoreFrom(Map<String, Object> m)")
    assert "cb.pin()" in rt and "batch.unpin()" in _method(rt, "public void shutdown()")
    cb = re.sub(r"/\*.*?\*/|//[^\n]*", "", _java("ColumnarBatch.java"), flags=re.S)
    assert "ShpNative.HOST_REGISTER.invokeExact(m, m.byteSize())" in cb
    ms = _method(cb, "void markStaged()")
    assert "staged.addLast(open)" in ms and "open = free.pollFirst()" in ms
    cs = _method(cb, "long commitStaged()")
    assert cs.index("staged.pollFirst()") < cs.index("commitRows(c)") < cs.index("decoded = c")
    for getter in ("int keyAt(long i)", "long tsAt(long i)", "int streamAt(long i)"):
        assert "decoded." in _method(cb, getter)
    # the narrow form (the mirror's narrow=True): 4-byte ts offsets from the batch's first ts, 2-byte ids
    assert "batch.narrowOk()" in st and "ShpNative.STAGE_BATCH_NARROW.invokeExact(engine, batch.descriptor()" in st
    assert "policy == FlushPolicy.PIPELINED && maxKeys <= 65536" in rt
    app = _method(cb, "void append(long timestamp, int keyId, int streamIndex, Object[] data)")
    assert "o.base = timestamp" in app and "if (d != (int) d)" in app and "o.wide = true" in app
    assert "o.key16.setAtIndex(JAVA_SHORT, n, (short) keyId)" in app
    assert "return narrow && open.n > 0 && !open.wide;" in _method(cb, "boolean narrowOk()")
