import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from diff_util import compare, per_key, program_for, run, small_stream
from oracle.oracle import OracleEngine
from siddhi_amd.native import HipEngine
q = int(sys.argv[1]); n = int(sys.argv[2]); keys = int(sys.argv[3]); batch = int(sys.argv[4])
cq = program_for(q)
g = small_stream(q, n, keys)
a = per_key(run(OracleEngine(cq.program_json(), 0), cq, g))
eng = HipEngine(cq.program_json(), 0, max_keys=keys, max_batch=max(batch, 1024))
print("path", eng.path, flush=True)
b = per_key(run(eng, cq, g, batch))
print("compare:", compare(a, b))
