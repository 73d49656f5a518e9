"""In-tree native build of dedloc_amd (gfx950 HIP kernels + torch.library bindings + C++ runtime).

The build is deliberately plain: every ``csrc/kernels/*.hip`` file is compiled by ``hipcc
--offload-arch=gfx950`` into its own object (fast: those translation units include only HIP
headers), ``csrc/bindings.cpp`` is the single translation unit that includes torch, and everything
is linked into ``dedloc_amd/_C.so`` next to this file, so the shared object travels with the
repository snapshot to the GPU box.  The control-plane server (``csrc/runtime``) is linked into a
separate ``dedloc_amd/_dht.so`` with no torch dependency.

Objects are rebuilt only when their source or any header is newer (mtime), so repeated calls are
cheap.  Run ``python -m dedloc_amd._build`` to build from the command line.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(os.path.dirname(ROOT), "build", "obj")
ARCH = os.environ.get("DEDLOC_OFFLOAD_ARCH", "gfx950")
SO_PATH = os.path.join(ROOT, "_C.so")
DHT_SO_PATH = os.path.join(ROOT, "_dht.so")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def _torch_paths():
    import torch
    import torch.utils.cpp_extension as ce

    abi = int(torch.compiled_with_cxx11_abi())
    return ce.include_paths(), ce.library_paths(), abi


def _newer(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build step failed ({r.returncode}):\n{' '.join(cmd)}\n{r.stdout}")
    return r.stdout


def build(verbose: bool = False, jobs: int | None = None) -> str:
    os.makedirs(BUILD, exist_ok=True)
    headers = glob.glob(os.path.join(CSRC, "include", "*.h"))
    # every header under csrc/ (comm/*.h, runtime/*.h, ...): a translation unit may include any of them
    all_headers = sorted(set(headers) | set(glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)))
    hip_srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    inc = ["-I", os.path.join(CSRC, "include")]
    hip_flags = ["--offload-arch=" + ARCH, *HIP_FLAGS]
    jobs = jobs or min(8, os.cpu_count() or 4)

    jobs_list = []
    objs = []
    for src in hip_srcs:
        obj = os.path.join(BUILD, os.path.basename(src).replace(".hip", ".o"))
        objs.append(obj)
        if _newer(obj, [src] + headers + [__file__]):
            jobs_list.append(["hipcc", *hip_flags, *FILE_FLAGS.get(os.path.basename(src), []), *inc, "-c", src,
                              "-o", obj])

    tinc, tlib, abi = _torch_paths()
    # translation units that include torch: the operator bindings and the RCCL data plane (csrc/comm)
    torch_srcs = [os.path.join(CSRC, "bindings.cpp")] + sorted(glob.glob(os.path.join(CSRC, "comm", "*.cpp")))
    for src in torch_srcs:
        name = os.path.basename(src).replace(".cpp", ".o")
        obj = os.path.join(BUILD, name if src.endswith("bindings.cpp") else "comm_" + name)
        objs.append(obj)
        if _newer(obj, [src] + all_headers):
            cmd = ["g++", "-O2", "-std=c++17", "-fPIC", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-D__HIP_PLATFORM_AMD__",
                   "-DUSE_ROCM", "-I", f"{ROCM}/include", *inc]
            for p in tinc:
                cmd += ["-I", p]
            cmd += ["-I", sysconfig.get_paths()["include"], "-c", src, "-o", obj]
            jobs_list.append(cmd)

    # host-side C++ that does not include torch
    for src in sorted(glob.glob(os.path.join(CSRC, "host", "*.cpp"))):
        obj = os.path.join(BUILD, "host_" + os.path.basename(src).replace(".cpp", ".o"))
        objs.append(obj)
        if _newer(obj, [src] + all_headers):
            jobs_list.append(["g++", "-O2", "-std=c++17", "-fPIC", "-Wall", "-D__HIP_PLATFORM_AMD__", "-I",
                              f"{ROCM}/include", *inc, "-c", src, "-o", obj])

    rt_srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    rt_objs = []
    for src in rt_srcs:
        obj = os.path.join(BUILD, "rt_" + os.path.basename(src).replace(".cpp", ".o"))
        rt_objs.append(obj)
        if _newer(obj, [src] + all_headers):
            jobs_list.append(["g++", "-O2", "-std=c++17", "-fPIC", "-Wall", *inc, "-c", src, "-o", obj])

    with cf.ThreadPoolExecutor(jobs) as ex:
        list(ex.map(lambda c: _run(c, verbose), jobs_list))

    if _newer(SO_PATH, objs):
        _link(objs, SO_PATH, tlib, verbose)
    if rt_objs and _newer(DHT_SO_PATH, rt_objs):
        _run(["g++", "-shared", "-fPIC", *rt_objs, "-o", DHT_SO_PATH, "-lpthread"], verbose)
    _OBJS[:] = objs
    return SO_PATH


_OBJS: list = []  # the kernel library's objects, in link order (filled by build)
HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=fast", "-munsafe-fp-atomics"]
# per-file extra flags (none at present: -fno-slp-vectorize on attention.hip, which keeps the softmax
# f32 arithmetic out of v_pk_*_f32, measured 2.5% slower in the backward and equal in the forward —
# profiles/r4_ab_attention_no_slp.jsonl)
FILE_FLAGS: dict = {}


def _link(objs, out, tlib, verbose):
    cmd = ["hipcc", "--offload-arch=" + ARCH, "-shared", "-fPIC", *objs, "-o", out]
    for p in tlib:
        cmd += ["-L", p, f"-Wl,-rpath,{p}"]
    # -lrccl resolves in torch's lib dir first: the same librccl.so.1 torch loads (one RCCL per process)
    cmd += ["-lc10", "-ltorch", "-ltorch_cpu", "-lc10_hip", "-ltorch_hip", "-lamdhip64", "-lrccl", "-L", f"{ROCM}/lib",
            f"-Wl,-rpath,{ROCM}/lib"]
    _run(cmd, verbose)


def build_variant(name: str, rev: str, kernels, verbose: bool = False, flags=None) -> str:
    """Measurement helper for same-box A/B runs: the kernel library with the given ``csrc/kernels``
    files taken from git revision ``rev`` (everything else as built now), linked into
    ``ab/_C_<name>.so``; a process loads it instead of ``_C.so`` with DEDLOC_NATIVE_LIB=<that path>."""
    build(verbose)
    vdir = os.path.join(os.path.dirname(BUILD), "variant_" + name)
    os.makedirs(vdir, exist_ok=True)
    repo = os.path.dirname(ROOT)
    swap = {}
    for k in kernels:
        src = os.path.join(vdir, os.path.basename(k))
        where = "" if k.endswith(".cpp") else "kernels/"  # bindings.cpp lives in csrc/ itself
        text = subprocess.run(["git", "-C", repo, "show", f"{rev}:dedloc_amd/csrc/{where}{os.path.basename(k)}"],
                              check=True, capture_output=True, text=True).stdout
        with open(src, "w") as f:
            f.write(text)
        if k.endswith(".cpp"):
            obj = src.replace(".cpp", ".o")
            tinc, _, abi = _torch_paths()
            cmd = ["g++", "-O2", "-std=c++17", "-fPIC", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-D__HIP_PLATFORM_AMD__",
                   "-DUSE_ROCM", "-I", f"{ROCM}/include", "-I", os.path.join(CSRC, "include")]
            for ip in tinc:
                cmd += ["-I", ip]
            _run(cmd + list(flags or []) + ["-I", sysconfig.get_paths()["include"], "-c", src, "-o", obj], verbose)
        else:
            obj = src.replace(".hip", ".o")
            extra = FILE_FLAGS.get(os.path.basename(k), []) if flags is None else list(flags)
            _run(["hipcc", "--offload-arch=" + ARCH, *HIP_FLAGS, *extra, "-I", os.path.join(CSRC, "include"), "-c",
                  src, "-o", obj], verbose)
        swap[os.path.basename(obj)] = obj
    out_dir = os.path.join(repo, "ab")
    os.makedirs(out_dir, exist_ok=True)
    out = os.path.join(out_dir, f"_C_{name}.so")
    objs = [swap.get(os.path.basename(o), o) for o in _OBJS]
    _link(objs, out, _torch_paths()[1], verbose)
    return out


if __name__ == "__main__":
    if len(sys.argv) > 3 and sys.argv[1] == "variant":  # python -m dedloc_amd._build variant NAME REV kernel.hip ...
        # [--flags="-fno-x -fy"]: compile the swapped files with these extra flags instead of FILE_FLAGS
        fl = [a for a in sys.argv[4:] if a.startswith("--flags=")]
        ks = [a for a in sys.argv[4:] if not a.startswith("--") and a != "-v"]
        print(build_variant(sys.argv[2], sys.argv[3], ks, verbose="-v" in sys.argv,
                            flags=fl[0][len("--flags="):].split() if fl else None))
    else:
        print(build(verbose="-v" in sys.argv))
