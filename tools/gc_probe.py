import sys, json
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/conjugate-gradient_amd")
import bench
out = bench.general_coefficients(20, 5)
for k, v in out.items():
    if isinstance(v, dict) and "value" in v:
        print(k, v["layout"][:40], v["value"], v["spmv_us"], v.get("own_bytes_frac"))
    else:
        print(k, v)
