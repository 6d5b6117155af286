"""set_matrix setup time of the C3 host CSR (DIA: host encode + code upload)."""
import sys, time
sys.path.insert(0, "conjugate-gradient_amd")
import numpy as np, cgx
rp, col, val = cgx.laplacian3d(216, 216, 216)
for i in range(3):
    with cgx.Solver(0) as s:
        t = time.perf_counter(); s.set_matrix(rp, col, val)
        i = s.info()
        print("set_matrix ms %.1f host %.1f dev %.1f layout %s" % (1e3*(time.perf_counter()-t), i["setup_host_ms"], i["setup_device_ms"], i["layout_name"]), flush=True)
