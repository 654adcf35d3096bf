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
    return sorted(set(re.findall(r"^\s*(?:int|void\*?|double|const char\*)\s+(shp_\w+)\s*\(", src, re.M)))


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


def test_config_struct_layout_matches_header():
    # shp_config: int32 device, int32 max_keys, int64 max_batch, int64 max_matches, int64 start_clock,
    # int32 force_general, int32 profile_kernels
    assert ctypes.sizeof(native.ShpConfig) == 40
    assert ctypes.sizeof(native.ShpBatch) == 48
    assert ctypes.sizeof(native.ShpMatches) == 72


def test_program_compiler_rejects_out_of_scope():
    from siddhi_amd.query.compiler import compile_app, SiddhiAppCreationException
    from siddhi_amd.query.siddhiql import SiddhiParserException
    with pytest.raises((SiddhiAppCreationException, SiddhiParserException)):
        compile_app("define stream S (a int); from every e1=S -> e2=S select * insert into O;")
