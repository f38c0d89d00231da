"""Build the native MI355X extension ``idc_models_amd/_idc_native*.so`` with hipcc (gfx950 only).

No torch.utils.cpp_extension / hipify: the kernels are plain HIP C++ written for CDNA4, the
bindings are pybind11, and the module has no libtorch dependency (tensors cross the boundary as
device pointers + the HIP stream handle), so it builds in seconds and loads in any process.

    python tools/build_native.py            # incremental
    python tools/build_native.py --clean
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build", "native")
PKG = os.path.join(ROOT, "idc_models_amd")
ARCH = os.environ.get("IDC_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

SOURCES = [
    "kernels/conv_igemm.hip",
    "kernels/conv_igemm_g0.hip",
    "kernels/conv_igemm_g1.hip",
    "kernels/conv_igemm_g2.hip",
    "kernels/conv_igemm_g3.hip",
    "kernels/conv_igemm_g4.hip",
    "kernels/conv_igemm_g5.hip",
    "kernels/conv_big.hip",
    "kernels/conv_img.hip",
    "kernels/conv_stem.hip",
    "kernels/wgrad_stem.hip",
    "kernels/conv_wgrad.hip", "kernels/wgrad_big.hip",
    "kernels/nn_kernels.hip",
    "kernels/pool_img.hip",
    "kernels/dwconv.hip",
    "kernels/dense_stage.hip",
    "kernels/dense_rows.hip",
    "kernels/dense_infer.hip",
    "kernels/mb_chain.hip",
    "kernels/mb_infer.hip",
    "kernels/dense_stage_bwd.hip",
    "kernels/dense_rows_bwd.hip",
    "kernels/mlp_head.hip",
    "kernels/secagg.hip",
    "comm/communicator.cpp",
    "runtime/plan.cpp",
    "runtime/guard_alloc.cpp",
]

# RCCL (= NCCL API on ROCm) for the native communicator.  Its soname is librccl.so.1, the same as
# the copy torch ships: in a process that imported torch first (the package always does) the loader
# reuses torch's already-mapped library, so one RCCL serves both communicators.
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
LINK_LIBS = [f"-L{ROCM}/lib", "-lrccl", f"-Wl,-rpath,{ROCM}/lib"]


def ext_path() -> str:
    return os.path.join(PKG, "_idc_native" + sysconfig.get_config_var("EXT_SUFFIX"))


def _headers():
    hs = []
    for d, _, fs in os.walk(CSRC):
        hs += [os.path.join(d, f) for f in fs if f.endswith(".h")]
    return hs


def _compile(src: str, extra) -> str:
    import pybind11

    s = os.path.join(CSRC, src)
    o = os.path.join(BUILD, src.replace("/", "_") + ".o")
    newest_dep = max([os.path.getmtime(s)] + [os.path.getmtime(h) for h in _headers()])
    if os.path.exists(o) and os.path.getmtime(o) >= newest_dep and not extra.get("force"):
        return o
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-c", s, "-o", o,
           f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}",
           "-Wno-unused-result", "-Wno-unused-variable"]
    # MFMA accumulators in the VGPR form: without it the register allocator keeps them in AGPRs ON
    # TOP of the kernel's VGPRs (unified register file), one occupancy step below what the kernel
    # needs -- e.g. the DenseNet concat-gradient dgrad tile 126 VGPRs + 16 AGPRs = 3 waves/SIMD,
    # 4 with this flag; 46 of the 552 conv tiles and the image-resident 3x3 data gradients (1 -> 2,
    # 2 -> 4 waves) gain, none spills (tools/kernel_resources.py, round 5)
    if not src.endswith(".cpp"):
        cmd += ["-mllvm", "-amdgpu-mfma-vgpr-form"]
    if src.endswith(".cpp"):
        cmd += ["-x", "hip"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr[-6000:]}")
    return o


H5_PREFIX = os.environ.get("IDC_HDF5_PREFIX", "/opt/conda")


def h5_ext_path() -> str:
    return os.path.join(PKG, "_idc_h5" + sysconfig.get_config_var("EXT_SUFFIX"))


def build_h5(verbose: bool = True):
    """Host-only pybind11 module over libhdf5 (Keras-layout weight files)."""
    import pybind11

    src = os.path.join(CSRC, "ckpt", "h5io.cpp")
    out = h5_ext_path()
    hdr = os.path.join(H5_PREFIX, "include", "hdf5.h")
    if not os.path.exists(hdr):
        if verbose:
            print(f"[build_native] libhdf5 not found under {H5_PREFIX}; HDF5 checkpoints disabled")
        return None
    if os.path.exists(out) and os.path.getmtime(out) >= os.path.getmtime(src):
        return out
    cmd = ["g++", "-O2", "-std=c++17", "-shared", "-fPIC", src, "-o", out,
           f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}",
           f"-I{H5_PREFIX}/include", f"-L{H5_PREFIX}/lib", "-lhdf5", f"-Wl,-rpath,{H5_PREFIX}/lib",
           # the rpath also exposes an older libstdc++ in that prefix: link ours statically
           "-static-libstdc++", "-static-libgcc"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"h5io build failed:\n{r.stderr[-4000:]}")
    if verbose:
        print(f"[build_native] {out}")
    return out


CONDA_PREFIX = os.environ.get("IDC_HOSTLIB_PREFIX", "/opt/conda")

# host-only pybind11 modules: (module name, source, include subdir, libs)
HOST_MODULES = [
    ("_idc_data", "data/loader.cpp", "libpng16", ["png16", "z"]),
    ("_idc_paillier", "fed/paillier_gmp.cpp", "", ["gmp"]),
]


def host_ext_path(name: str) -> str:
    return os.path.join(PKG, name + sysconfig.get_config_var("EXT_SUFFIX"))


def build_host_module(name: str, src_rel: str, inc_sub: str, libs, verbose: bool = True):
    """g++ build of a host-only pybind11 module against libraries of the image's /opt/conda
    prefix (rpath'd; libstdc++ linked statically because that prefix ships an older one)."""
    import pybind11

    src = os.path.join(CSRC, src_rel)
    out = host_ext_path(name)
    inc = os.path.join(CONDA_PREFIX, "include", inc_sub) if inc_sub else os.path.join(CONDA_PREFIX, "include")
    if not os.path.isdir(inc):
        if verbose:
            print(f"[build_native] {inc} not found; {name} disabled")
        return None
    if os.path.exists(out) and os.path.getmtime(out) >= os.path.getmtime(src):
        return out
    # the module's own include dir only (not all of /opt/conda/include, which carries headers that
    # would shadow the system's)
    cmd = ["g++", "-O3", "-std=c++17", "-shared", "-fPIC", "-pthread", src, "-o", out + ".tmp",
           f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}", f"-I{inc}",
           f"-L{CONDA_PREFIX}/lib"] + [f"-l{l}" for l in libs] + [
           f"-Wl,-rpath,{CONDA_PREFIX}/lib", "-static-libstdc++", "-static-libgcc"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"{name} build failed:\n{r.stderr[-4000:]}")
    os.replace(out + ".tmp", out)
    if verbose:
        print(f"[build_native] {out}")
    return out


SANITIZERS = {
    # host code only (no GPU sanitizer on this pool): the threaded PNG loader / pinned ring, the
    # GMP Paillier vector ops and the libhdf5 weight I/O
    "address": ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"],
    "thread": ["-fsanitize=thread"],
}


SONAMES = {"gmp": "libgmp.so.10", "hdf5": "libhdf5.so.103", "png16": "libpng16.so.16", "z": "libz.so.1"}


def sanitize_dir(kind: str) -> str:
    return os.path.join(ROOT, "build", "sanitize", kind)


def build_sanitized(kind: str, verbose: bool = True) -> str:
    """Instrumented builds of every host-only module into build/sanitize/<kind>/ (loaded through
    IDC_HOST_EXT_DIR, utils/hostext.py).  libstdc++ is linked dynamically here: the sanitizer
    runtimes must intercept its allocator."""
    import pybind11

    out_dir = sanitize_dir(kind)
    os.makedirs(out_dir, exist_ok=True)
    # the image's /opt/conda/lib also carries an OLDER sanitizer runtime (libasan.so.5): an rpath
    # to that prefix would map it beside the system runtime the test process preloads (two ASan
    # shadows -> abort), so the instrumented modules rpath a directory holding only the libraries
    # they need from the prefix
    libdir = os.path.join(out_dir, "lib")
    os.makedirs(libdir, exist_ok=True)
    for so in SONAMES.values():
        src_so, dst = os.path.join(CONDA_PREFIX, "lib", so), os.path.join(libdir, so)
        if os.path.exists(src_so) and not os.path.lexists(dst):
            os.symlink(os.path.realpath(src_so), dst)
    mods = list(HOST_MODULES) + [("_idc_h5", "ckpt/h5io.cpp", "", ["hdf5"])]
    for name, src_rel, inc_sub, libs in mods:
        src = os.path.join(CSRC, src_rel)
        out = os.path.join(out_dir, name + sysconfig.get_config_var("EXT_SUFFIX"))
        if os.path.exists(out) and os.path.getmtime(out) >= os.path.getmtime(src):
            continue
        inc = os.path.join(CONDA_PREFIX, "include", inc_sub) if inc_sub else os.path.join(CONDA_PREFIX, "include")
        cmd = (["g++", "-O1", "-g", "-fno-omit-frame-pointer", "-std=c++17", "-shared", "-fPIC", "-pthread"]
               + SANITIZERS[kind] + [src, "-o", out, f"-I{pybind11.get_include()}",
                                     f"-I{sysconfig.get_paths()['include']}", f"-I{inc}", f"-L{libdir}"]
               + [f"-l:{SONAMES[l]}" for l in libs] + [f"-Wl,-rpath,{libdir}"])
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"{name} ({kind} sanitizer) build failed:\n{r.stderr[-4000:]}")
        if verbose:
            print(f"[build_native] {out}")
    return out_dir


def build(clean: bool = False, jobs: int = 8, verbose: bool = True) -> str:
    build_h5(verbose)
    for name, src, inc, libs in HOST_MODULES:
        if os.path.exists(os.path.join(CSRC, src)):
            build_host_module(name, src, inc, libs, verbose)
    if clean and os.path.isdir(BUILD):
        shutil.rmtree(BUILD)
    os.makedirs(BUILD, exist_ok=True)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, {}), SOURCES))
    out = ext_path()
    if not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(o) for o in objs):
        tmp = out + ".tmp"
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs + LINK_LIBS
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-4000:]}")
        os.replace(tmp, out)
    if verbose:
        print(f"[build_native] {out}")
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--sanitize", choices=sorted(SANITIZERS), default=None,
                    help="build the host-only modules with a sanitizer into build/sanitize/<kind>/")
    a = ap.parse_args()
    if a.sanitize:
        build_sanitized(a.sanitize)
    else:
        build(a.clean, a.j)
