"""Debug aid: the ct4 golden stream's batch 0 on the GPU against the fixture,
printing the first mismatching packets with their columns."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

from cilium_amd import synth  # noqa: E402
from test_gpu_ct import _golden_engine, _run  # noqa: E402

g = np.load(os.path.join(ROOT, "tests", "golden", "ct4.npz"))
e = _golden_engine(g)
for k, v in zip(g["pre_keys"], g["pre_vals"]):
    assert e.ct4_update(k, v) == 0
t = {k[2:]: g[k] for k in g.files if k.startswith("t_")}
sl = slice(int(g["cuts"][0]), int(g["cuts"][1]))
tb = {k: x[sl] for k, x in t.items()}
v, cr, idt, st = _run(torch, e, tb, int(g["nows"][0]))
bad = np.nonzero((v != g["b_verdict"][sl]) | (cr != g["b_ct_ret"][sl]) | (idt != g["b_identity"][sl]))[0]
print("n", len(v), "bad", len(bad))
for i in bad[:40]:
    print(i, {k: int(tb[k][i]) for k in ("saddr", "daddr", "sport", "dport", "proto", "l4b", "flags", "ep")},
          "got", int(v[i]), int(cr[i]), int(idt[i]), int(st[i]),
          "want", int(g["b_verdict"][sl][i]), int(g["b_ct_ret"][sl][i]), int(g["b_identity"][sl][i]),
          int(g["b_stage"][sl][i]))
