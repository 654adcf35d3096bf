/*
 * ProgramInfo — what the host reads back from a lowered program (shp_compile_siddhiql's JSON): the
 * stream names in program["streams"] order (receiver stream index), program["columns"] (the SoA
 * columns a batch carries: stream index, attribute position, type) and, per state in
 * MetaStateEvent order (program["states"][i]["id"] = StateInputStreamParser's stateIndex,
 * core/util/parser/StateInputStreamParser.java:177), its stream, its reference id (e1, ...) and
 * whether it is a count state (multi-valued, :380-403).  A minimal JSON reader for that fixed
 * document; the engine itself parses the program (siddhi_amd/csrc/compile.h).
 * Source only: no JDK in this repository's image (DESIGN.md §6).
 */
package io.siddhi.core.query.input.stream.state.gpu;

import java.util.ArrayList;
import java.util.LinkedHashMap;
import java.util.List;
import java.util.Map;

final class ProgramInfo {

    final String[] streams;
    final ColumnarBatch.Column[] columns;
    final boolean partitioned;
    final int[] stateStream;        // per state id: index into streams
    final String[] stateRef;        // per state id: the reference id (e1, ...), null when none
    final boolean[] stateMulti;     // per state id: a count state (multi-valued slot)
    final int countMax;             // the largest <min:max> bound (CHAIN32: a chain's longest length)
    final boolean timers;           // an absent state (`not S for T`): the query has a Scheduler

    private ProgramInfo(String[] streams, ColumnarBatch.Column[] columns, boolean partitioned, int[] stateStream,
                        String[] stateRef, boolean[] stateMulti, int countMax, boolean timers) {
        this.streams = streams;
        this.columns = columns;
        this.partitioned = partitioned;
        this.stateStream = stateStream;
        this.stateRef = stateRef;
        this.stateMulti = stateMulti;
        this.countMax = countMax;
        this.timers = timers;
    }

    @SuppressWarnings("unchecked")
    static ProgramInfo parse(String json) {
        Map<String, Object> p = (Map<String, Object>) new Reader(json).value();
        List<Object> ss = (List<Object>) p.get("streams");
        String[] names = new String[ss.size()];
        for (int i = 0; i < names.length; i++) {
            names[i] = (String) ((Map<String, Object>) ss.get(i)).get("name");
        }
        List<Object> cs = (List<Object>) p.get("columns");
        ColumnarBatch.Column[] cols = new ColumnarBatch.Column[cs.size()];
        for (int i = 0; i < cols.length; i++) {
            Map<String, Object> c = (Map<String, Object>) cs.get(i);
            String t = (String) c.get("type");
            char tag = "int".equals(t) ? 'i' : "long".equals(t) ? 'l' : "float".equals(t) ? 'f'
                    : "double".equals(t) ? 'd' : "bool".equals(t) ? 'b' : 's';
            cols[i] = new ColumnarBatch.Column(((Number) c.get("stream")).intValue(),
                    ((Number) c.get("attr")).intValue(), tag);
        }
        List<Object> st = (List<Object>) p.get("states");
        int[] sst = new int[st.size()];
        String[] sref = new String[st.size()];
        boolean[] smulti = new boolean[st.size()];
        boolean timers = false;
        for (Object o : st) {
            Map<String, Object> m = (Map<String, Object>) o;
            int id = ((Number) m.get("id")).intValue();
            sst[id] = ((Number) m.get("stream")).intValue();
            sref[id] = (String) m.get("ref");
            timers |= Boolean.TRUE.equals(m.get("absent"));
        }
        int cmax = markCounts(p.get("tree"), smulti);
        return new ProgramInfo(names, cols, Boolean.TRUE.equals(p.get("partitioned")), sst, sref, smulti, cmax,
                timers);
    }

    // the states under a "count" node of program["tree"] (CountStateElement: multiValue = true);
    // returns the largest count bound ("max") in the tree
    @SuppressWarnings("unchecked")
    private static int markCounts(Object node, boolean[] multi) {
        if (!(node instanceof Map)) {
            return 0;
        }
        Map<String, Object> n = (Map<String, Object>) node;
        int mx = 0;
        if ("count".equals(n.get("t")) && n.get("state") instanceof Number) {
            multi[((Number) n.get("state")).intValue()] = true;
            mx = n.get("max") instanceof Number ? ((Number) n.get("max")).intValue() : 0;
        }
        for (Object v : n.values()) {
            if (v instanceof Map) {
                mx = Math.max(mx, markCounts(v, multi));
            }
        }
        return mx;
    }

    private static final class Reader {
        private final String s;
        private int i;

        Reader(String s) {
            this.s = s;
        }

        private void ws() {
            while (i < s.length() && Character.isWhitespace(s.charAt(i))) {
                i++;
            }
        }

        Object value() {
            ws();
            char c = s.charAt(i);
            if (c == '{') {
                Map<String, Object> m = new LinkedHashMap<>();
                i++;
                ws();
                if (s.charAt(i) == '}') {
                    i++;
                    return m;
                }
                while (true) {
                    ws();
                    String k = string();
                    ws();
                    i++;  // ':'
                    m.put(k, value());
                    ws();
                    if (s.charAt(i++) == '}') {
                        return m;
                    }
                }
            }
            if (c == '[') {
                List<Object> a = new ArrayList<>();
                i++;
                ws();
                if (s.charAt(i) == ']') {
                    i++;
                    return a;
                }
                while (true) {
                    a.add(value());
                    ws();
                    if (s.charAt(i++) == ']') {
                        return a;
                    }
                }
            }
            if (c == '"') {
                return string();
            }
            if (s.startsWith("true", i)) {
                i += 4;
                return Boolean.TRUE;
            }
            if (s.startsWith("false", i)) {
                i += 5;
                return Boolean.FALSE;
            }
            if (s.startsWith("null", i)) {
                i += 4;
                return null;
            }
            int b = i;
            while (i < s.length() && "+-0123456789.eEINaity".indexOf(s.charAt(i)) >= 0) {
                i++;
            }
            String num = s.substring(b, i);
            return num.matches("-?\\d+") ? (Object) Long.parseLong(num) : (Object) Double.parseDouble(num);
        }

        private String string() {
            StringBuilder o = new StringBuilder();
            i++;  // opening quote
            while (s.charAt(i) != '"') {
                char c = s.charAt(i++);
                if (c == '\\') {
                    char e = s.charAt(i++);
                    switch (e) {
                        case 'n': o.append('\n'); break;
                        case 't': o.append('\t'); break;
                        case 'r': o.append('\r'); break;
                        case 'b': o.append('\b'); break;
                        case 'f': o.append('\f'); break;
                        case 'u': o.append((char) Integer.parseInt(s.substring(i, i + 4), 16)); i += 4; break;
                        default: o.append(e); break;
                    }
                } else {
                    o.append(c);
                }
            }
            i++;
            return o.toString();
        }
    }
}
