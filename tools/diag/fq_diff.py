"""Diagnostic: where does the HIP fake-quant differ from the reference FakeQuantize golden?"""
import json, os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "velocity-asr_amd")]
import torch
from velocity_asr import ops
z = np.load(os.path.join(REPO, "tests/golden/int8_b2_3s.npz"))
x = z["fq_x"]
for name, kw in json.loads(str(z["fq_cases"])):
    bits, sym = kw["bits"], kw["symmetric"]
    qmin, qmax = ((-(2 ** (bits - 1)), 2 ** (bits - 1) - 1) if sym else (0, 2 ** bits - 1))
    s, zp = z[f"fq_{name}__scale"], z[f"fq_{name}__zp"]
    y = ops.fakequant(torch.from_numpy(x).cuda(), torch.from_numpy(np.array(s)).cuda(),
                      torch.from_numpy(np.array(zp)).cuda(), qmin, qmax).cpu().numpy()
    g = z[f"fq_{name}__y"]
    bad = np.argwhere(y.view(np.int32) != g.view(np.int32))
    print(name, "mismatches", len(bad))
    for r, c in bad[:6]:
        ss = s.reshape(-1)[r if s.size > 1 else 0]
        zz = zp.reshape(-1)[r if zp.size > 1 else 0]
        t = np.float32(x[r, c]) / np.float32(ss)
        print("  x=%r s=%r zp=%r x/s=%r t=%r got=%r want=%r" % (x[r, c], ss, zz, t, np.float32(t + zz), y[r, c], g[r, c]))
