"""Minimal driver for rocprofv3 PMC passes: config-2 tables, one 64M-tuple
batch resident in HBM, 3 classify launches (variant from CGPU_CLASSIFY_VARIANT)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from cilium_amd import synth  # noqa: E402
from cilium_amd.engine import Engine  # noqa: E402

cfg = synth.CONFIGS[os.environ.get("CGPU_PMC_CONFIG", "gpu")]
n = int(os.environ.get("CGPU_PMC_TUPLES", cfg["n_tuples"]))
T = synth.make_tables(**cfg)
t = synth.make_tuples(T, n)
e = Engine(device=0, **T.engine_config())
synth.load_engine(e, T)
e.commit()
d = synth.to_device(t)
out = {"verdict": torch.empty(n, dtype=torch.int32, device="cuda"),
       "identity": torch.empty(n, dtype=torch.int32, device="cuda"), "stage": None}
for _ in range(3):
    e.classify_v4(d, out=out)
torch.cuda.synchronize()
print("ok", n)
