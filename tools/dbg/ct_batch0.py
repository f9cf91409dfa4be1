"""Diagnostic: batch 0 of test_ct_stream_vs_restatement, GPU vs restatement."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "oracle"))
import numpy as np
import torch
from cilium_amd import synth
from cilium_amd.engine import Engine
from oracle import Oracle

T = synth.make_tables(**synth.CONFIGS["cpu"])
t, lb, sl = synth.make_ct_workload(T, 60_000, mean_pkts=10.0, span=0.05)
n = len(t["saddr"]) // 3
tb = {k: v[:n] for k, v in t.items()}
o = Oracle(**T.oracle_config()); synth.load_oracle(o, T); synth.load_lxc(o, sl); o.ct_set_max(1 << 18)
v0, cr0, i0, s0, _ = o.classify_v4_ct(tb, 1000)
e = Engine(device=0, **T.engine_config(), ct_max=1 << 18)
synth.load_engine(e, T); synth.load_lxc(e, sl); e.commit()
out = e.classify_v4_ct(synth.to_device(tb), 1000)
torch.cuda.synchronize()
v = out["verdict"].cpu().numpy(); cr = out["ct_ret"].cpu().numpy()
bad = np.nonzero((v != v0) | (cr != cr0))[0]
print("sort bits", os.environ.get("CGPU_CT_SORT_BITS"), "chunk env", os.environ.get("CGPU_CT_CHUNK"), "mismatch", len(bad), "of", n,
      "gpu count", e.ct4_count(), "oracle count", o.ct4_count())
for i in bad[:10]:
    sa, da = tb["saddr"][i], tb["daddr"][i]
    same = np.nonzero(((tb["saddr"] == sa) & (tb["daddr"] == da)) | ((tb["saddr"] == da) & (tb["daddr"] == sa)))[0]
    print(i, v[i], v0[i], cr[i], cr0[i], tb["proto"][i], tb["flags"][i], tb["l4b"][i], "pair pkts", len(same),
          "pos", int(np.searchsorted(same, i)))
print("gpu -155:", (v == -155).sum(), "oracle -155:", (v0 == -155).sum())
