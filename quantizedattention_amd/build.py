"""Build libqattn.so (all HIP kernels + the C-ABI) in-tree for gfx950.

Plain hipcc, no torch headers: the library is a C-ABI boundary (include/qattn.h) that any host
(ctypes here) binds.  Objects are rebuilt when a source, a header or this file (the flags) is newer
than the object.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
INCLUDE = PKG.parent / "include"
BUILD = PKG / "_build"
LIB = PKG / "libqattn.so"
DEV_LIB = PKG / "libqattn_dev.so"   # fragment-layout probes (csrc/dev): tests only, not product API
OPS_LIB = PKG / "libqattn_torch.so"  # TORCH_LIBRARY(qattn) operators over libqattn.so (csrc/torch)
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
CFLAGS = [
    "-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}",
    "-fhip-fp32-correctly-rounded-divide-sqrt",  # the quantiser needs IEEE fp32 division
    "-fno-gpu-rdc", "-Wno-unused-result", f"-I{INCLUDE}",
]

# Per-source extras.  The bf16 forward keeps its fp32 softmax scalar (-fno-slp-vectorize: the SLP
# vectoriser otherwise emits v_pk_mul/add_f32, which issue through the matrix pipe and wait ~38
# cycles behind a co-resident wave's MFMA, tools/ubench) and runs with IEEE mode off
# (-mno-amdgpu-ieee, valid with -fno-honor-nans: no NaN reaches it), so v_max needs no canonicalising
# v_max x,x of its bit-cast inputs.
FILE_FLAGS = {
    "bf16_fwd.hip": ["-fno-slp-vectorize", "-mno-amdgpu-ieee", "-fno-honor-nans"],
    "bf16_bwd.hip": ["-fno-slp-vectorize"],
    # The JVP forward (one wave per SIMD, 4 fp32 accumulator sets) needs more than 256 registers:
    # by default hipcc gives the MFMAs AGPR accumulators and copies all 128 of them to VGPRs at every
    # loop iteration for the (rare) rescale; the VGPR form keeps them in VGPRs and moves the Q
    # fragments to AGPRs instead (287 instead of 534 vector instructions per 64 keys).
    "jvp_fwd.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1", "-mllvm", "-amdgpu-sched-strategy=max-ilp"],
    # The int8 forward under the max-ilp machine scheduler: same code, ordered for latency; no spill
    # in any instantiation, bit-identical outputs, -1.2 % non-causal and -1.5 to -3 % causal at
    # config 3 (profiles/r05_int8_fwd_sched_ab.log).  (iterative-ilp spills here; max-ilp spills the
    # dK+dV kernel, and the bf16 forward does not move under either.)
    "int8_attn_fwd.hip": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"],
    # the same scheduler for the JVP forward (config 5: 0.270-0.272 against 0.276 ms) and the MX-FP4
    # forward (536-544 against 545-559 us); the bf16 backward is slower under it (3.85 against 3.79-3.83
    # ms) and keeps the default (profiles/r05_int8_fwd_sched_ab.log)
    "mxfp4_attn.hip": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"],
}


def _compile(src: Path, obj: Path) -> str:
    cmd = [HIPCC, *CFLAGS, *FILE_FLAGS.get(src.name, []), "-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stderr}")
    return src.name


STAMP = BUILD / "source_hash"
VERSION_SRC = BUILD / "qattn_version.cpp"


def _version_object(digest: str, verbose: bool) -> Path:
    """The generated qattn_abi_version() / qattn_source_hash() of include/qattn.h."""
    src = (f'#include "qattn.h"\n'
           f'extern "C" int qattn_abi_version(void) {{ return QATTN_ABI_VERSION; }}\n'
           f'extern "C" const char* qattn_source_hash(void) {{ return "{digest}"; }}\n')
    obj = BUILD / "qattn_version.o"
    if not obj.exists() or not VERSION_SRC.exists() or VERSION_SRC.read_text() != src:
        VERSION_SRC.write_text(src)
        cmd = [HIPCC, "-O2", "-std=c++17", "-fPIC", f"-I{INCLUDE}", "-c", str(VERSION_SRC), "-o", str(obj)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {VERSION_SRC.name}:\n{r.stderr}")
        if verbose:
            print(f"[qattn build] compiled {VERSION_SRC.name}", file=sys.stderr)
    return obj


def build(verbose: bool = True, jobs: int = 8) -> Path:
    from ._srchash import library_hash
    BUILD.mkdir(exist_ok=True)
    digest = library_hash()
    # a change of sources or flags rebuilds every object, whatever the file times say (a tree copied
    # to another machine may carry any mtimes)
    force = not STAMP.exists() or STAMP.read_text().strip() != digest
    ver = _version_object(digest, verbose)
    _build_lib(sorted(CSRC.glob("*.hip")), LIB, "", verbose, jobs, force, extra=[ver])
    _build_lib(sorted((CSRC / "dev").glob("*.hip")), DEV_LIB, "dev_", verbose, jobs, force)
    STAMP.write_text(digest + "\n")
    build_torch_ops(verbose)
    build_c_host(verbose)
    return LIB


C_HOST_SRC = PKG.parent / "tests" / "c_abi" / "int8_step.cpp"
C_HOST_BIN = PKG.parent / "tests" / "c_abi" / "int8_step"


def build_c_host(verbose: bool = True) -> Path | None:
    """tests/c_abi/int8_step: a host program of the C ABI alone (no torch, no Python), linked to
    libqattn.so through the $ORIGIN-relative rpath; tests/test_gpu_c_abi.py runs it."""
    if not C_HOST_SRC.exists():
        return None
    deps = [C_HOST_SRC, LIB] + list(INCLUDE.glob("*.h"))
    if C_HOST_BIN.exists() and C_HOST_BIN.stat().st_mtime >= max(d.stat().st_mtime for d in deps):
        return C_HOST_BIN
    cmd = [HIPCC, "-O2", "-std=c++17", f"--offload-arch={ARCH}", f"-I{INCLUDE}", str(C_HOST_SRC),
           "-o", str(C_HOST_BIN) + ".tmp", f"-L{PKG}", "-lqattn",
           "-Wl,-rpath,$ORIGIN/../../quantizedattention_amd"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        # a test program, not part of the library: its link failing must not fail the build
        # (tests/test_gpu_c_abi.py, which needs it, reports the missing program)
        print(f"[qattn build] warning: C host program not built:\n{r.stderr}", file=sys.stderr)
        return None
    os.replace(str(C_HOST_BIN) + ".tmp", C_HOST_BIN)
    if verbose:
        print(f"[qattn build] linked {C_HOST_BIN}", file=sys.stderr)
    return C_HOST_BIN


def build_torch_ops(verbose: bool = True) -> Path:
    """libqattn_torch.so: the C++ operator layer (csrc/torch/qattn_ops.cpp), host code only, compiled
    against torch's headers and linked to libqattn.so (found beside it through the $ORIGIN rpath)."""
    import torch
    srcs = sorted((CSRC / "torch").glob("*.cpp"))
    deps = srcs + [LIB] + list(INCLUDE.glob("*.h"))
    if OPS_LIB.exists() and OPS_LIB.stat().st_mtime >= max(d.stat().st_mtime for d in deps):
        return OPS_LIB
    tdir = Path(torch.__file__).resolve().parent
    cmd = [os.environ.get("CXX", "g++"), "-O2", "-std=c++17", "-fPIC", "-shared",
           "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
           f"-D_GLIBCXX_USE_CXX11_ABI={int(torch._C._GLIBCXX_USE_CXX11_ABI)}",
           f"-I{tdir / 'include'}", f"-I{tdir / 'include' / 'torch' / 'csrc' / 'api' / 'include'}",
           "-I/opt/rocm/include", f"-I{INCLUDE}", *map(str, srcs), "-o", str(OPS_LIB) + ".tmp",
           f"-L{tdir / 'lib'}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
           f"-L{PKG}", "-lqattn", "-Wl,-rpath,$ORIGIN"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"torch operator library build failed:\n{r.stderr}")
    os.replace(str(OPS_LIB) + ".tmp", OPS_LIB)
    if verbose:
        print(f"[qattn build] linked {OPS_LIB}", file=sys.stderr)
    return OPS_LIB


def _build_lib(srcs, lib, prefix: str, verbose: bool, jobs: int, force: bool = False,
               extra=()) -> None:
    BUILD.mkdir(exist_ok=True)
    # (this file too: it holds the compile flags)
    headers = list(CSRC.glob("*.h")) + list(INCLUDE.glob("*.h")) + [Path(__file__)]
    hdr_mtime = max((h.stat().st_mtime for h in headers), default=0.0)
    todo = []
    objs = []
    for s in srcs:
        o = BUILD / (prefix + s.stem + ".o")
        objs.append(o)
        if force or not o.exists() or o.stat().st_mtime < max(s.stat().st_mtime, hdr_mtime):
            todo.append((s, o))
    objs += list(extra)
    if todo:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            for name in ex.map(lambda so: _compile(*so), todo):
                if verbose:
                    print(f"[qattn build] compiled {name}", file=sys.stderr)
    if todo or not lib.exists() or lib.stat().st_mtime < max(o.stat().st_mtime for o in objs):
        tmp = lib.with_suffix(".so.tmp")
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp), *map(str, objs)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
        os.replace(tmp, lib)
        if verbose:
            print(f"[qattn build] linked {lib}", file=sys.stderr)


if __name__ == "__main__":
    build()
