"""debug: MIN stream decode, engine vs oracle, first differing var record field by field"""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
from minpaxos_amd import _lib
_lib.load()
import numpy as np
from minpaxos_amd import records as R, wire as W
from minpaxos_amd.engine import Engine
from oracle_lib import Oracle
from test_stream_decode import kat_stream
for proto in (0, 1):
    e, o = Engine(0, 5, proto), Oracle(5, proto)
    for name, b in (("kat", kat_stream(proto)),
                    ("rand", W.random_stream(proto, np.random.default_rng(3), 300, p_var=0.3))):
        g, w = e.decode_stream(b), o.decode_stream(b)
        print(proto, name, "res", {f: (int(g[4][f]), int(w[4][f])) for f in R.STREAM_RESULT.names})
        for k, nm in enumerate(("ar", "prep", "var", "oth")):
            if len(g[k]) != len(w[k]) or g[k].tobytes() != w[k].tobytes():
                for i in range(min(len(g[k]), len(w[k]))):
                    if g[k][i].tobytes() != w[k][i].tobytes():
                        print("  ", nm, i, "got", g[k][i], "want", w[k][i])
                        break
                print("  ", nm, "lens", len(g[k]), len(w[k]))
