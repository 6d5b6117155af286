"""Sequences of fresh in-process C4 groups in ONE process:
  python tools/c4_diag3.py f8:10 u8:10 ...   (f/u: fused on/off, P, maxit)
prints the reflection asymmetry of x (b = 1: zero up to rounding) and x[0]."""
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "conjugate-gradient_amd"))
sys.path.insert(0, str(REPO / "tests"))
import cgx  # noqa: E402
from test_gpu_fullsize import c4_group  # noqa: E402  (the full-size test's group builder)

for tok in sys.argv[1:]:
    kind, rest = tok[0], tok[1:]
    P, m = (int(v) for v in rest.split(":"))
    its, x, h, st = c4_group(cgx.CGX_ALG_HS, kind == "f", m, P=P)
    print(f"{tok}: its={its} fused={[s['fused'] for s in st][:2]} "
          f"asym={float(np.abs(x - x[::-1]).max()):.3e} x[0]={x[0]!r} h[-1]={h[-1]!r}", flush=True)
