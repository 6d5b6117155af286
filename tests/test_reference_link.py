"""The op-level drop-in claim of INTEGRATION.md section 1, checked in the
build container: the reference's own cg.c (rnelias/Conjugate-Gradient,
unmodified, read where it lies under /root/reference) compiles against
include/mv_ops.h and links against libcgx.so in place of mv_ops.c, its
mv_mult / dot_product / sv_mult / vec_add / vec_sub / new_mv_struct* calls
resolving to libcgx.  Compile and link only (running it needs a GPU); the
objects go to a temporary directory, nothing is copied into the repo and
nothing travels to the GPU box.  Skipped where /root/reference is absent."""
import os
import shutil
import subprocess
import tempfile
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
REF = Path("/root/reference")
LIB = REPO / "conjugate-gradient_amd" / "lib"

pytestmark = pytest.mark.skipif(not (REF / "cg.c").exists() or shutil.which("gcc") is None,
                                reason="needs /root/reference/cg.c and gcc (build container)")

MV_OPS = ["new_mv_struct", "new_mv_struct_with_size", "free_mv_struct", "mv_deep_copy",
          "dot_product", "sv_mult", "mv_mult", "vec_add", "vec_sub"]


def test_unmodified_cg_c_links_against_libcgx():
    with tempfile.TemporaryDirectory() as td:
        td = Path(td)
        # a symlink, so `#include "mv_ops.h"` is searched beside the link (not
        # beside the reference's own header) and then in include/
        os.symlink(REF / "cg.c", td / "cg.c")
        obj, exe = td / "cg.o", td / "cg"
        subprocess.run(["gcc", "-Wall", "-g", "-I", str(REPO / "include"), "-c", str(td / "cg.c"),
                        "-o", str(obj)], check=True, capture_output=True)
        undef = subprocess.run(["nm", "-u", str(obj)], check=True, capture_output=True,
                               text=True).stdout.split()
        called = [s for s in MV_OPS if s in undef]
        assert {"mv_mult", "dot_product", "sv_mult", "vec_add", "vec_sub"} <= set(called)
        subprocess.run(["gcc", "-o", str(exe), str(obj), f"-L{LIB}", "-lcgx",
                        f"-Wl,-rpath,{LIB}"], check=True, capture_output=True)
        # every mv_ops symbol cg.c uses is bound to libcgx at run time
        dyn = subprocess.run(["nm", "-D", "--defined-only", str(LIB / "libcgx.so")], check=True,
                             capture_output=True, text=True).stdout.split()
        assert all(s in dyn for s in called)
        needed = subprocess.run(["readelf", "-d", str(exe)], check=True, capture_output=True,
                                text=True).stdout
        assert "libcgx.so" in needed
