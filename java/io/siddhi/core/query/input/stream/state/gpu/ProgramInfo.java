/*
 * ProgramInfo — what the host reads back from a lowered program (shp_compile_siddhiql's JSON): the
 * stream names in program["streams"] order (receiver stream index) and program["columns"] (the
 * SoA columns a batch carries: stream index, attribute position, type).  A minimal JSON reader for
 * that fixed document; the engine itself parses the program (siddhi_amd/csrc/compile.h).
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

    private ProgramInfo(String[] streams, ColumnarBatch.Column[] columns, boolean partitioned) {
        this.streams = streams;
        this.columns = columns;
        this.partitioned = partitioned;
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
        return new ProgramInfo(names, cols, Boolean.TRUE.equals(p.get("partitioned")));
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
