import sys
sys.path.insert(0, "conjugate-gradient_amd"); sys.path.insert(0, "tests")
import torch  # noqa: F401
import numpy as np
import cgx
import helpers as H
for dim, (nx, ny, nz) in [(3, (12, 12, 12)), (3, (7, 5, 9)), (2, (32, 32, 1))]:
    host = cgx.laplacian3d(nx, ny, nz) if dim == 3 else cgx.laplacian2d(nx, ny)
    with cgx.Solver(0) as s:
        s.gen_laplacian(dim, nx, ny, nz)
        inf = s.info()
        print("gen", dim, (nx, ny, nz), "n", inf["n"], "nnz", inf["nnz"], "host nnz", len(host[1]), flush=True)
        rp, col, val = s.matrix()
        print(" rp eq", np.array_equal(rp, host[0]), "col eq", np.array_equal(col, host[1]),
              "val eq", np.array_equal(val, host[2]), flush=True)
        if not np.array_equal(col, host[1]):
            d = np.nonzero(col != host[1])[0][:5]
            print(" first col diffs", d, col[d], host[1][d], flush=True)
    n = nx * ny * nz
    x = np.random.default_rng(5).standard_normal(n)
    with cgx.Solver(0) as s:
        s.set_stencil(dim, nx, ny, nz)
        print("stencil nnz", s.info()["nnz"], flush=True)
        y = s.spmv(x)
    yr = H.o_spmv(*host, x)
    print(" stencil eq", np.array_equal(y, yr), np.max(np.abs(y - yr)), flush=True)
