"""Build the in-tree native extension ``unet_distributed_amd/_C*.so`` for gfx950.

Every ``csrc/kernels/*.hip`` translation unit is compiled with
``hipcc --offload-arch=gfx950`` and the pybind11 bindings/executor
(``csrc/runtime/*.cpp``) with hipcc as host code; all objects are linked into
one shared library next to the package so it travels with the repository
snapshot to the GPU box (a JIT cache under ~/.cache would not).

Incremental: an object is rebuilt only when the hash of its source, the
shared headers and the flags changes.  ``python -m unet_distributed_amd.native.build``.
"""

import concurrent.futures as cf
import glob
import hashlib
import os
import subprocess
import sys
import sysconfig

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(PKG, "csrc")
OBJDIR = os.path.join(os.path.dirname(PKG), "build", "native")
ARCH = os.environ.get("UNET_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def ext_suffix():
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def so_path():
    return os.path.join(PKG, "_C" + ext_suffix())


def _includes():
    import pybind11
    return ["-I" + pybind11.get_include(), "-I" + sysconfig.get_paths()["include"],
            "-I" + os.path.join(CSRC, "kernels"), "-I" + os.path.join(CSRC, "runtime")]


COMMON = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
          "-Wno-unused-variable", "-Wno-unused-but-set-variable"]


# every kernel TU is built once per 16-bit element type (common.h): bf16 in namespace
# `unet`, fp16 in namespace `unet_f16`
VARIANTS = {"bf16": [], "f16": ["-DUNET_FP16", "-Dunet=unet_f16"]}


def _hash(path, flags):
    h = hashlib.sha256()
    h.update(" ".join(flags).encode())
    for f in sorted(glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True) +
                    glob.glob(os.path.join(CSRC, "**", "*.inc"), recursive=True)):
        h.update(open(f, "rb").read())
    h.update(open(path, "rb").read())
    return h.hexdigest()[:20]


def _compile(job):
    src, variant = job
    is_hip = src.endswith(".hip")
    flags = COMMON + _includes()
    if is_hip:
        flags = flags + ["--offload-arch=" + ARCH, "-munsafe-fp-atomics"] + VARIANTS[variant]
    else:
        flags = flags + ["-x", "c++", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include"]
    key = _hash(src, flags)
    obj = os.path.join(OBJDIR, os.path.basename(src) + "." + variant + "." + key + ".o")
    if os.path.exists(obj):
        return obj, False
    cmd = [HIPCC] + flags + ["-c", src, "-o", obj + ".tmp"]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("compile failed: %s\n%s" % (" ".join(cmd), r.stdout))
    os.replace(obj + ".tmp", obj)
    return obj, True


def _check_kernel_stubs(so):
    """Every launched kernel's host stub must be defined in the library: clang can drop a
    kernel's stub silently (e.g. a lambda call inside a target builtin's argument list),
    which only surfaces as an undefined symbol when the extension is imported."""
    import shutil
    nm = shutil.which("nm") or shutil.which("llvm-nm")
    if nm is None:
        return
    r = subprocess.run([nm, "-u", "-C", so], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    bad = [ln.strip() for ln in r.stdout.splitlines() if "__device_stub__" in ln]
    if bad:
        raise RuntimeError("undefined kernel stubs in %s:\n%s" % (so, "\n".join(bad[:20])))


def build(verbose=True, jobs=None):
    os.makedirs(OBJDIR, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")) +
                  glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    # (f32*.hip: fp32 kernels, element-type independent -- the bf16 build only)
    work = [(f, v) for f in srcs
            for v in (VARIANTS if f.endswith(".hip") and not os.path.basename(f).startswith("f32") else ["bf16"])]
    # costliest TUs first so the pool finishes together (the row-window conv units are
    # small files that instantiate conv_win.h's ~150 kernels)
    work.sort(key=lambda j: -(os.path.getsize(j[0]) + (10 ** 6 if "conv_win" in j[0] else 0)))
    jobs = jobs or min(8, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(jobs) as ex:
        results = list(ex.map(_compile, work))
    objs = [r[0] for r in results]
    rebuilt = any(r[1] for r in results)
    out = so_path()
    # the link manifest names the objects the current .so was built from: a cached
    # object set that differs (e.g. after reverting a source) must be relinked even
    # though no object is newer than the library
    manifest = os.path.join(OBJDIR, "link_manifest.txt")
    want = "\n".join(sorted(os.path.basename(o) for o in objs))
    have = open(manifest).read() if os.path.exists(manifest) else ""
    if rebuilt or not os.path.exists(out) or want != have or any(
            os.path.getmtime(o) > os.path.getmtime(out) for o in objs):
        cmd = [HIPCC, "-shared", "-fPIC", "--offload-arch=" + ARCH] + objs + ["-o", out + ".tmp"]
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed: %s\n%s" % (" ".join(cmd), r.stdout))
        _check_kernel_stubs(out + ".tmp")
        os.replace(out + ".tmp", out)
        with open(manifest, "w") as f:
            f.write(want)
        if verbose:
            print("built", out)
    elif verbose:
        print("up to date", out)
    return out


if __name__ == "__main__":
    build()
    sys.exit(0)
