"""tools/isa_check.py: the build step that keeps `s_waitcnt vmcnt(0)` out of the hot kernels' loops."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import isa_check  # noqa: E402

TEXT = """
0000000000001000 <k_a>:
\ts_load_dwordx2 s[0:1], s[4:5], 0x0                    // 000000001000: C0060002 00000000
\ts_waitcnt vmcnt(0)                                       // 000000001008: BF8C0F70
\tglobal_load_dword v1, v[2:3], off                        // 00000000100C: DC508000 017F0002
\ts_waitcnt vmcnt(0) lgkmcnt(0)                            // 000000001014: BF8C0070
\ts_cbranch_scc1 3                                         // 000000001018: BF850003 <k_a+0x28>
\ts_waitcnt vmcnt(0)                                       // 00000000101C: BF8C0F70
\ts_cbranch_vccnz 65530                                    // 000000001020: BF87FFFA <k_a+0x10>
\ts_branch 65527                                           // 000000001024: BF82FFF7 <k_a+0x8>
\ts_endpgm                                                 // 000000001028: BF810000
"""


def test_loop_detection_on_a_synthetic_listing():
    r = isa_check.loop_waits(TEXT)
    inloop, nested, total, loops = r["k_a"]
    # loops: [0x1010, 0x1020] and [0x1008, 0x1024]; waits at 0x1008 (outer), 0x1014 and 0x101C (both)
    assert (inloop, nested, total, loops) == (3, 2, 3, 2)


@pytest.mark.skipif(not os.path.exists(os.path.join(isa_check.OBJ, "sweep_lean.o")), reason="library not built here")
def test_built_kernels_within_budget():
    assert isa_check.main([]) == 0
