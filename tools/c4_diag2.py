"""C4/8 in-process group, the test's exact sequence (fresh group, one run of
maxit 10): fused vs unfused, and the reflection symmetry of x (b = 1)."""
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "conjugate-gradient_amd"))
sys.path.insert(0, str(REPO / "tests"))
import cgx  # noqa: E402
from test_gpu_fullsize import c4_group  # noqa: E402


def sym(x):
    return float(np.abs(x - x[::-1]).max())


for rep in range(2):
    out = {}
    for fused in (True, False):
        its, x, h, st = c4_group(cgx.CGX_ALG_HS, fused, int(sys.argv[1]) if len(sys.argv) > 1 else 10)
        out[fused] = x
        print(f"rep {rep} fused={fused} its={its} asym={sym(x):.3e} x[0]={x[0]!r}", flush=True)
    d = np.abs(out[True] - out[False])
    bad = np.nonzero(d > 0)[0]
    print(f"rep {rep}: fused vs unfused max diff {d.max():.3e}, {len(bad)} rows differ, "
          f"first {bad[:5].tolist()} last {bad[-5:].tolist()}", flush=True)
