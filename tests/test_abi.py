"""CPU checks of the C-ABI boundary: libsiddhi_hip.so loads and exports every symbol
declared in include/siddhi_hip.h (no compute calls: there is no GPU here)."""
import ctypes
import os
import re

import pytest

from siddhi_amd import native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "siddhi_hip.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|int32_t|int64_t|void\*?|double|const char\*|shp_engine\*|shp_dict\*)\s+(shp_\w+)\s*\(", src, re.M)))


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ("shp_engine_create", "shp_push_batch", "shp_advance_clock", "shp_engine_destroy", "shp_last_error"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    if not os.path.exists(native.LIB_PATH):
        pytest.fail("libsiddhi_hip.so not built (python -m siddhi_amd.build)")
    L = ctypes.CDLL(native.LIB_PATH)
    for s in declared_symbols():
        assert hasattr(L, s), s
    assert sorted(native.SYMBOLS) == declared_symbols()


def _c_layout():
    """sizeof/offsetof of the ABI structs as the C compiler lays them out from the header."""
    import subprocess
    import tempfile
    fields = {"shp_config": [f[0] for f in native.ShpConfig._fields_],
              "shp_batch": [f[0] for f in native.ShpBatch._fields_],
              "shp_matches": [f[0] for f in native.ShpMatches._fields_]}
    body = []
    for st, fs in fields.items():
        body.append(f'printf("{st} %zu", sizeof({st}));')
        for f in fs:
            body.append(f'printf(" %zu", offsetof({st}, {f}));')
        body.append('printf("\\n");')
    src = ("#include <stdio.h>\n#include <stddef.h>\n#include \"siddhi_hip.h\"\nint main(void){"
           + "".join(body) + "return 0;}")
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "l.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "l")
        subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), "-o", exe, c])
        out = subprocess.check_output([exe]).decode().split("\n")
    res = {}
    for line in out:
        if line.strip():
            parts = line.split()
            res[parts[0]] = [int(x) for x in parts[1:]]
    return res


def test_struct_layouts_match_header():
    lay = _c_layout()
    for name, cls in (("shp_config", native.ShpConfig), ("shp_batch", native.ShpBatch),
                      ("shp_matches", native.ShpMatches)):
        size, *offs = lay[name]
        assert ctypes.sizeof(cls) == size, name
        assert [getattr(cls, f[0]).offset for f in cls._fields_] == offs, name


def test_program_compiler_rejects_out_of_scope():
    from siddhi_amd.query.compiler import compile_app, SiddhiAppCreationException
    from siddhi_amd.query.siddhiql import SiddhiParserException
    with pytest.raises((SiddhiAppCreationException, SiddhiParserException)):
        compile_app("define stream S (a int); from every e1=S -> e2=S select * insert into O;")
