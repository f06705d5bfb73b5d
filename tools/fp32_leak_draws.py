#!/usr/bin/env python3
"""float32 model (tools/fp32_model.py) of the leakage-only draws of tests/test_gpu_floor.py: the
kernel's error / the port's error per draw for three forms of forward pass 2's twiddles (the
three-term recurrence, six exactly rounded anchors, the exactly rounded table of all powers).
Output: profiles/r05/parity/fp32_model_leak_draws.txt."""
import sys, json, numpy as np
import os
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, 'tools'), os.path.join(R, 'tests')]
import fp32_model as M
from oracle import oracle as O
from extio_sddc_amd.synth import make_stream
import test_gpu_floor as T
H = O.filter_bank(1.0); H32 = O.filter_bank(1.0, np.float32)
rows = []
for d, tb, lsb, nblk, seed in T._leak_draws():
    x = make_stream(nblk, "bench", seed=seed)
    ex = O.r2iq(x, nblk, d, tb, lsb, 0, H=H)
    port = O.max_rel_err(O.r2iq(x, nblk, d, tb, lsb, 0, dtype=np.float32, H=H32), ex)
    r = {"d": d, "tb": tb, "lsb": lsb, "seed": seed, "port": port}
    for name, kw in [("kernel", {}), ("anchor6", {"twmode": "anchor6"}), ("table", {"twmode": "table"})]:
        r[name] = O.max_rel_err(M.r2iq_model(x, nblk, d, tb, lsb, 0, H[d], **kw), ex) / port
    rows.append(r)
    print(json.dumps(r), flush=True)
for k in ("kernel", "anchor6", "table"):
    v = np.array([r[k] for r in rows])
    print(k, "geomean %.3f max %.3f n>1.2: %d" % (np.exp(np.log(v).mean()), v.max(), (v > 1.2).sum()))
