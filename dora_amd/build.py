"""Builds the in-tree native artefacts with hipcc for gfx950 (no CMake, no JIT cache).

    python -m dora_amd.build            # libdora_gpu.so + tools
Outputs land in dora_amd/lib/ (git-ignored, but shipped to the GPU box by gpurun).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "dora_amd", "csrc")
OBJ = os.path.join(ROOT, "build", "obj")
LIB = os.path.join(ROOT, "dora_amd", "lib")
INCLUDE = os.path.join(ROOT, "include")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
ARCH = "gfx950"

LIB_SOURCES = ["runtime.cpp", "plan.cpp", "device_array.cpp", "kernels.hip", "shm.cpp", "bcast.cpp", "operator_api.cpp", "stdout_capture.cpp",
               "wire.cpp", "trace.cpp", "daemon.cpp", "node.cpp", "aql.cpp", "interdaemon.cpp",
               "bincode.cpp"]
AQL_KERNELS = "aql_kernels.hip"  # standalone gfx950 code object embedded in the library
LIB_NAME = "libdora_gpu.so"

CXXFLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wextra", "-Wno-unused-parameter",
            f"-I{INCLUDE}", f"-I{CSRC}"]


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _headers():
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    hs += [os.path.join(INCLUDE, f) for f in os.listdir(INCLUDE) if f.endswith(".h")]
    hs.append(os.path.abspath(__file__))
    return hs


def _compile(src, obj, verbose):
    if src.endswith(".hip"):
        cmd = [HIPCC, "-x", "hip", f"--offload-arch={ARCH}", *CXXFLAGS, "-c", src, "-o", obj]
    else:
        cmd = [HIPCC, "-x", "c++", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", *CXXFLAGS, "-c", src, "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


def _compile_all(sources, verbose):
    os.makedirs(OBJ, exist_ok=True)
    heads = _headers()
    objs = []
    for s in sources:
        src = os.path.join(CSRC, s)
        obj = os.path.join(OBJ, s.replace("/", "_") + ".o")
        if _newer(obj, [src, *heads]):
            _compile(src, obj, verbose)
        objs.append(obj)
    return objs


def _aql_blob(verbose):
    """The AQL pack kernels as a raw gfx950 code object (no offload bundle), wrapped into an
    object file with .incbin (symbols dora_aql_code_object[_end], aql.cpp)."""
    os.makedirs(OBJ, exist_ok=True)
    src = os.path.join(CSRC, AQL_KERNELS)
    co = os.path.join(OBJ, "aql_kernels.co")
    if _newer(co, [src, *_headers()]):
        # kernel-argument preload: the single-segment kernels take all 56 B of arguments in
        # SGPRs (the struct-argument kernels are not affected: their preload length stays 0)
        cmd = [HIPCC, "--genco", f"--offload-arch={ARCH}", "--offload-device-only",
               "--no-gpu-bundle-output", "-O3", "-std=c++17", "-mllvm",
               "-amdgpu-kernarg-preload-count=14", f"-I{INCLUDE}", f"-I{CSRC}", src, "-o", co]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    asm = os.path.join(OBJ, "aql_blob.S")
    with open(asm, "w") as f:
        f.write(".section .rodata\n.p2align 12\n.globl dora_aql_code_object\n"
                "dora_aql_code_object:\n"
                f'.incbin "{co}"\n'
                ".globl dora_aql_code_object_end\ndora_aql_code_object_end:\n"
                '.section .note.GNU-stack,"",@progbits\n')
    obj = os.path.join(OBJ, "aql_blob.o")
    if _newer(obj, [co]):
        cmd = [HIPCC, "-c", "-x", "assembler-with-cpp", asm, "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    return obj


def build(verbose: bool = False) -> str:
    os.makedirs(LIB, exist_ok=True)
    objs = _compile_all(LIB_SOURCES, verbose) + [_aql_blob(verbose)]
    out = os.path.join(LIB, LIB_NAME)
    if _newer(out, objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out, *objs,
               "-Wl,-soname," + LIB_NAME, "-L/opt/rocm/lib", "-lhsa-runtime64", "-ldl", "-lpthread",
               "-lrt"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    return out


TESTING_SOURCES = ["testing/testing.cpp"]
TESTING_NAME = "libdora_gpu_testing.so"


def build_testing(verbose: bool = False) -> str:
    """libdora_gpu_testing.so: the test and microbenchmark hooks (include/dora_gpu_testing.h),
    linked against libdora_gpu.so (rpath $ORIGIN) — the shipped library exports none of them."""
    lib = build(verbose)
    objs = _compile_all(TESTING_SOURCES, verbose)
    out = os.path.join(LIB, TESTING_NAME)
    if _newer(out, objs + [lib]):
        cmd = [HIPCC, "-shared", "-fPIC", "-o", out, *objs, f"-L{LIB}", "-ldora_gpu",
               "-Wl,-rpath,$ORIGIN", "-Wl,-soname," + TESTING_NAME]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    return out


TOOLS = {  # binary name -> sources (linked against libdora_gpu.so, rpath $ORIGIN)
    "dora-gpu-daemon": ["tools/daemon_main.cpp"],
    "dora-gpu-bench-sink": ["tools/bench_sink.cpp"],
    "dora-gpu-relay": ["tools/relay.cpp"],
    "dora-gpu-bench-source": ["tools/bench_source.cpp"],
    "dora-gpu-runtime": ["tools/runtime_main.cpp"],
}


def build_tools(verbose: bool = False):
    out = []
    lib = build(verbose)
    for name, srcs in TOOLS.items():
        objs = _compile_all(srcs, verbose)
        exe = os.path.join(LIB, name)
        if _newer(exe, objs + [lib]):
            cmd = [HIPCC, f"--offload-arch={ARCH}", "-o", exe, *objs, f"-L{LIB}", "-ldora_gpu",
                   "-Wl,-rpath,$ORIGIN", "-ldl", "-lpthread", "-lrt"]
            if verbose:
                print(" ".join(cmd), flush=True)
            subprocess.run(cmd, check=True)
        out.append(exe)
    return out


PYEXT_SOURCE = "pyext.cpp"


def build_pyext(verbose: bool = False) -> str:
    """dora_amd/_dora_node<EXT_SUFFIX>: the Python node's per-send path as a CPython extension
    (the reference's Python node is a native PyO3 module), linked against libdora_gpu.so in
    dora_amd/lib (rpath $ORIGIN/lib) so it shares the library ctypes loads."""
    import sysconfig
    lib = build(verbose)
    inc = sysconfig.get_paths()["include"]
    os.makedirs(OBJ, exist_ok=True)
    src = os.path.join(CSRC, PYEXT_SOURCE)
    obj = os.path.join(OBJ, "pyext.cpp.o")
    if _newer(obj, [src, *_headers()]):
        cmd = [HIPCC, "-x", "c++", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", *CXXFLAGS,
               f"-I{inc}", "-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    out = os.path.join(ROOT, "dora_amd", "_dora_node" + sysconfig.get_config_var("EXT_SUFFIX"))
    if _newer(out, [obj, lib]):
        cmd = [HIPCC, "-shared", "-fPIC", "-o", out, obj, f"-L{LIB}", "-ldora_gpu",
               "-Wl,-rpath,$ORIGIN/lib"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    return out


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
    print(build_pyext(verbose="-v" in sys.argv))
    print(build_tools(verbose="-v" in sys.argv))
    print(build_testing(verbose="-v" in sys.argv))
