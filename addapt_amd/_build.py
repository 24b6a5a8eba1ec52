"""In-tree build of the native libraries (hipcc for gfx950, g++ for host C++).

Outputs land in addapt_amd/_lib/ (git-ignored, shipped to the GPU box with the
snapshot).  Rebuilds only when a source is newer than its output.
"""
import glob
import os
import subprocess
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
HOSTSRC = os.path.join(HERE, "host")
OUT = os.path.join(HERE, "_lib")
OBJ = os.path.join(OUT, "obj")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

GPU_SOURCES = ["kernels.hip", "mfe_cells.hip", "mfe_pair.hip", "outside_cells.hip", "pf_cells.hip", "pf_ring.hip", "outside_ring.hip", "adx_api.cpp",
               "energy.cpp"]


def _newer(src_list, out):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(s) > t for s in src_list)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed: %s\n%s" % (" ".join(cmd), r.stdout))
    return r.stdout


def build_gpu(force=False):
    os.makedirs(OBJ, exist_ok=True)
    lib = os.path.join(OUT, "libaddapt_gpu.so")
    # generated shape blocks (*.inc) are included by the kernels: a change must rebuild them
    headers = (glob.glob(os.path.join(CSRC, "*.hpp")) + glob.glob(os.path.join(CSRC, "*.inc")) +
               [os.path.join(ROOT, "include", "addapt_gpu.h")])
    jobs = []
    objs = []
    for src in GPU_SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(OBJ, src + ".o")
        objs.append(o)
        if force or _newer([s] + headers, o):
            jobs.append([HIPCC, "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-Wall",
                         "-Wno-unused-function", "-c", s, "-o", o])
    with ThreadPoolExecutor(max_workers=4) as ex:
        list(ex.map(_run, jobs))
    if force or jobs or not os.path.exists(lib):
        _run([HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", lib] + objs)
    return lib


def build_host(force=False):
    """C++ mirror of addapt's Device / ScoreFunction / MonteCarlo API + CLI."""
    srcs = sorted(glob.glob(os.path.join(HOSTSRC, "*.cc")))
    if not srcs:
        return None
    os.makedirs(OBJ, exist_ok=True)
    inc = os.path.join(ROOT, "include")
    headers = (glob.glob(os.path.join(inc, "addapt", "*.hh")) + [os.path.join(inc, "addapt_gpu.h")] +
               glob.glob(os.path.join(HOSTSRC, "*.hh")))
    lib = os.path.join(OUT, "libaddapt_host.so")
    lib_srcs = [s for s in srcs if not os.path.basename(s).startswith("app_")]
    if force or _newer(lib_srcs + headers, lib):
        _run(["g++", "-std=c++17", "-O2", "-fPIC", "-shared", "-Wall", "-I", inc, "-I", HOSTSRC,
              "-o", lib] + lib_srcs + ["-L", OUT, "-laddapt_gpu", "-ldl", "-Wl,-rpath,$ORIGIN"])
    for app in [s for s in srcs if os.path.basename(s).startswith("app_")]:
        exe = os.path.join(OUT, os.path.basename(app)[4:-3])
        if force or _newer([app, lib] + headers, exe):
            _run(["g++", "-std=c++17", "-O2", "-Wall", "-I", inc, "-o", exe, app, "-L", OUT,
                  "-laddapt_host", "-laddapt_gpu", "-Wl,-rpath,$ORIGIN"])
    return lib


def build_all(force=False):
    build_gpu(force)
    build_host(force)
