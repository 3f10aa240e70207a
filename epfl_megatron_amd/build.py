"""Ahead-of-time build of the native extensions (no JIT, no hipify).

* ``epfl_megatron_amd/_C.so``  — gfx950 HIP kernels (``csrc/*.hip``, compiled by
  ``hipcc --offload-arch=gfx950``) + pybind11/ATen bindings (``csrc/bindings.cpp``).
* ``epfl_megatron_amd/data/_helpers.so`` — CPU dataset index builders
  (``csrc/data_helpers.cpp``, g++ + pybind11).

Both land in-tree so they travel with the repository snapshot to the GPU box.
Usage: ``python -m epfl_megatron_amd.build [--force] [--jobs N]``.
"""
import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
BUILD = os.path.join(os.path.dirname(PKG), "build", "csrc")
ARCH = os.environ.get("EMA_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _torch_paths():
    import torch
    import torch.utils.cpp_extension as ce
    inc = ce.include_paths()
    lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}")
    return r.stdout


def build_kernels(force=False, jobs=None):
    os.makedirs(BUILD, exist_ok=True)
    headers = glob.glob(os.path.join(CSRC, "*.h"))
    hip_srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    inc, lib, abi = _torch_paths()
    common = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", CSRC,
              "-mcode-object-version=5", "-Wno-unused-result"]
    jobs_list = []
    objs = []
    for src in hip_srcs:
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _newer(obj, [src] + headers):
            jobs_list.append([HIPCC, "-c", src, "-o", obj] + common)
    # host-side sources that use ATen / pybind11 / hipBLASLt
    for bsrc in (os.path.join(CSRC, "bindings.cpp"), os.path.join(CSRC, "gemm_lt.cpp")):
        bobj = os.path.join(BUILD, os.path.basename(bsrc) + ".o")
        objs.append(bobj)
        if not (force or _newer(bobj, [bsrc] + headers)):
            continue
        cmd = [HIPCC, "-c", bsrc, "-o", bobj, "-O2", "-std=c++17", "-fPIC", "-I", CSRC,
               f"--offload-arch={ARCH}",
               f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_EXTENSION_NAME=_C",
               "-DTORCH_API_INCLUDE_EXTENSION_H", "-DUSE_ROCM=1", "-D__HIP_PLATFORM_AMD__=1",
               "-I", sysconfig.get_paths()["include"], "-Wno-unused-result",
               "-Wno-deprecated-declarations"]
        for i in inc:
            cmd += ["-I", i]
        jobs_list.append(cmd)
    n = jobs or int(os.environ.get("MAX_JOBS", os.cpu_count() or 4))
    with cf.ThreadPoolExecutor(max_workers=max(1, min(n, 16))) as ex:
        list(ex.map(_run, jobs_list))
    out = os.path.join(PKG, "_C.so")
    if force or jobs_list or not os.path.exists(out):
        _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", out] + objs +
             ["-L", lib, "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
              "-ltorch_python", f"-Wl,-rpath,{lib}", "-L/opt/rocm/lib", "-lhipblaslt",
             "-Wl,-rpath,/opt/rocm/lib"])
    return out


def build_data_helpers(force=False):
    import pybind11
    src = os.path.join(CSRC, "data_helpers.cpp")
    out = os.path.join(PKG, "data", "_helpers.so")
    if not os.path.exists(src):
        return None
    if force or _newer(out, [src]):
        _run(["g++", "-O3", "-shared", "-std=c++17", "-fPIC", "-I", pybind11.get_include(),
              "-I", sysconfig.get_paths()["include"], src, "-o", out])
    return out


def build_dedup(force=False):
    """``data/_dedup.so``: MinHash/LSH corpus de-duplication (CPU, g++)."""
    import pybind11
    src = os.path.join(CSRC, "dedup.cpp")
    out = os.path.join(PKG, "data", "_dedup.so")
    if force or _newer(out, [src]):
        _run(["g++", "-O3", "-shared", "-std=c++17", "-fPIC", "-pthread", "-I",
              pybind11.get_include(), "-I", sysconfig.get_paths()["include"], src, "-o", out])
    return out


SANITIZERS = {
    "asan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"],
    "tsan": ["-fsanitize=thread"],
}


def build_sanitized(kind, out_dir):
    """Host-sanitizer harness: ``data_helpers.cpp`` + ``dedup.cpp`` as embedded
    pybind11 modules linked with libpython into one executable
    (``csrc/sanitize_main.cpp``), instrumented with ``kind`` in
    :data:`SANITIZERS`.  The sanitizer runtime lives in the executable, so
    nothing is preloaded.  CPU code only (no GPU sanitizer on this pool)."""
    import pybind11
    os.makedirs(out_dir, exist_ok=True)
    flags = ["-O1", "-g", "-fno-omit-frame-pointer", "-std=c++17", "-pthread",
             "-DEMA_EMBEDDED", "-I", pybind11.get_include(),
             "-I", sysconfig.get_paths()["include"]] + SANITIZERS[kind]
    objs = []
    for src in ("data_helpers.cpp", "dedup.cpp", "sanitize_main.cpp"):
        o = os.path.join(out_dir, f"{kind}_{src}.o")
        _run(["g++", "-c"] + flags + [os.path.join(CSRC, src), "-o", o])
        objs.append(o)
    exe = os.path.join(out_dir, f"helpers_{kind}")
    libdir = sysconfig.get_config_var("LIBDIR")
    ver = sysconfig.get_config_var("LDVERSION")
    _run(["g++"] + SANITIZERS[kind] + ["-pthread", "-o", exe] + objs +
         [f"-L{libdir}", f"-lpython{ver}", "-ldl", "-lm", f"-Wl,-rpath,{libdir}"])
    return exe


def build_lab(force=False):
    """Bench-only GEMM lab (``scripts/lab``): ``scripts/lab/_gemm_lab.so``.
    Not part of ``build_all``: nothing in the framework loads it."""
    lab = os.path.join(os.path.dirname(PKG), "scripts", "lab")
    out = os.path.join(lab, "_gemm_lab.so")
    srcs = [os.path.join(lab, "gemm_lab.hip"), os.path.join(lab, "lab_bindings.cpp")]
    headers = glob.glob(os.path.join(CSRC, "*.h"))
    if not (force or _newer(out, srcs + headers)):
        return out
    inc, lib, abi = _torch_paths()
    objs = []
    for src in srcs:
        obj = os.path.join(BUILD, "lab_" + os.path.basename(src) + ".o")
        cmd = [HIPCC, "-c", src, "-o", obj, "-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}",
               "-I", CSRC, "-Wno-unused-result"]
        if src.endswith(".cpp"):
            cmd += [f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_EXTENSION_NAME=_gemm_lab",
                    "-DTORCH_API_INCLUDE_EXTENSION_H", "-DUSE_ROCM=1", "-D__HIP_PLATFORM_AMD__=1",
                    "-I", sysconfig.get_paths()["include"], "-Wno-deprecated-declarations"]
            for i in inc:
                cmd += ["-I", i]
        else:
            cmd += ["-mcode-object-version=5"]
        os.makedirs(BUILD, exist_ok=True)
        _run(cmd)
        objs.append(obj)
    _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", out] + objs +
         ["-L", lib, "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
          "-ltorch_python", f"-Wl,-rpath,{lib}"])
    return out


def build_all(force=False, jobs=None):
    build_dedup(force)
    h = build_data_helpers(force)
    k = build_kernels(force, jobs)
    return k, h


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=None)
    ap.add_argument("--only", choices=["kernels", "data"], default=None)
    ap.add_argument("--lab", action="store_true", help="also build the bench-only GEMM lab")
    a = ap.parse_args()
    if a.lab:
        print(build_lab(a.force))
    if a.only == "data":
        print(build_data_helpers(a.force))
    elif a.only == "kernels":
        print(build_kernels(a.force, a.jobs))
    else:
        print(build_all(a.force, a.jobs))


if __name__ == "__main__":
    sys.exit(main())
