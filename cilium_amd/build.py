"""Build cilium_amd/libl7gpu.so (HIP kernels for gfx950 + C++ host code).

Every translation unit is compiled with hipcc; the shared object is linked
against the libamdhip64.so that PyTorch-ROCm loads (torch/lib), so a process
that uses both torch (device memory, streams, torch.distributed/RCCL) and this
library runs exactly one HIP runtime.  Output stays in-tree so it travels to
the GPU box with the repo snapshot.
"""
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "build")
LIB = os.path.join(HERE, "libl7gpu.so")
LIB_TIMING = os.path.join(HERE, "libl7gpu_timing.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("L7G_ARCH", "gfx950")

COMMON = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", "-Wno-sign-compare"]
HIP_FLAGS = [f"--offload-arch={ARCH}", "-mcode-object-version=5", "-munsafe-fp-atomics"]


def torch_libdir():
    import importlib.util
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.submodule_search_locations:
        return None
    d = os.path.join(list(spec.submodule_search_locations)[0], "lib")
    return d if os.path.exists(os.path.join(d, "libamdhip64.so")) else None


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "**", "*.cc"), recursive=True) +
                  glob.glob(os.path.join(CSRC, "**", "*.hip"), recursive=True))


def headers():
    return glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True) + \
        glob.glob(os.path.join(HERE, "..", "include", "*.h"))


def _compile(src, obj, newest_header, defines=()):
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(src), newest_header):
        return None
    os.makedirs(os.path.dirname(obj), exist_ok=True)
    if src.endswith(".hip"):
        cmd = [HIPCC] + COMMON + HIP_FLAGS + list(defines) + ["-c", src, "-o", obj]
    else:  # host-only C++: plain g++ against the HIP runtime headers
        cmd = ["g++"] + COMMON + ["-I/opt/rocm/include", "-D__HIP_PLATFORM_AMD__"] + list(defines) + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return src


def build(verbose=False, jobs=8, timing=False, variant=None, defines=()):
    """timing=True builds the profiling variant libl7gpu_timing.so (kernels
    compiled with -DL7G_PHASE_TIMING; see l7g_debug_phase_times).  variant=NAME
    builds libl7gpu_NAME.so with extra -D defines (kernel experiments only;
    the product is always libl7gpu.so)."""
    if not variant and not timing and defines:
        # the product is built from its sources as they stand: a -D define could
        # only reach it through an experiment, and none may change a verdict
        raise ValueError("libl7gpu.so takes no -D defines; build a variant (variant=NAME) for experiments")
    srcs = sources()
    newest_header = max([os.path.getmtime(h) for h in headers()] + [0])
    if timing:
        variant, defines = "timing", ("-DL7G_PHASE_TIMING",) + tuple(defines)
    bdir = BUILD + ("_" + variant if variant else "")
    lib = os.path.join(HERE, f"libl7gpu_{variant}.so") if variant else LIB
    defines = tuple(defines)
    objs = [os.path.join(bdir, os.path.relpath(s, CSRC)) + ".o" for s in srcs]
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        done = list(ex.map(lambda so: _compile(so[0], so[1], newest_header, defines), zip(srcs, objs)))
    rebuilt = [d for d in done if d]
    if verbose and rebuilt:
        print("compiled:", *[os.path.relpath(r, HERE) for r in rebuilt], file=sys.stderr)
    LIB_OUT = lib
    if rebuilt or not os.path.exists(LIB_OUT) or os.path.getmtime(LIB_OUT) < max(os.path.getmtime(o) for o in objs):
        tl = torch_libdir()
        link = ["g++", "-shared", "-o", LIB_OUT + ".tmp"] + objs
        if tl:
            link += [f"-L{tl}", "-l:libamdhip64.so", f"-Wl,-rpath,{tl}"]
        else:
            link += ["-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib"]
        link += ["-pthread"]
        r = subprocess.run(link, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(link)}\n{r.stdout}\n{r.stderr}")
        os.replace(LIB_OUT + ".tmp", LIB_OUT)
    if not variant:
        # proxylib drop-in name: Envoy's Go filter dlopen()s "libcilium.so"
        # (pkg/envoy/server.go:227); it binds the five proxylib symbols.
        alias = os.path.join(HERE, "libcilium.so")
        if not os.path.islink(alias) or os.readlink(alias) != os.path.basename(LIB_OUT):
            if os.path.lexists(alias):
                os.remove(alias)
            os.symlink(os.path.basename(LIB_OUT), alias)
    return LIB_OUT


def build_test_natives(verbose=False):
    """tests/native/*.cc -> tests/native/bin/<name>: C++ drivers of the C-ABI
    headers (e.g. include/l7gpu_envoy.hpp), linked against libl7gpu.so."""
    lib = build(verbose=verbose)
    root = os.path.dirname(HERE)
    out = []
    for src in sorted(glob.glob(os.path.join(root, "tests", "native", "*.cc"))):
        name = os.path.splitext(os.path.basename(src))[0]
        exe = os.path.join(root, "tests", "native", "bin", name)
        deps = [src, lib] + headers()
        if not os.path.exists(exe) or os.path.getmtime(exe) < max(os.path.getmtime(d) for d in deps):
            os.makedirs(os.path.dirname(exe), exist_ok=True)
            cmd = ["g++", "-O2", "-std=c++17", "-Wall", "-I" + os.path.join(root, "include"), src, "-o", exe + ".tmp",
                   "-L" + HERE, "-l:libl7gpu.so", "-Wl,-rpath,$ORIGIN/../../../cilium_amd", "-pthread"]
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
            os.replace(exe + ".tmp", exe)
        out.append(exe)
    return out


if __name__ == "__main__":
    # python -m cilium_amd.build [--timing] [--variant NAME -DX=Y ...]
    argv = sys.argv[1:]
    var = argv[argv.index("--variant") + 1] if "--variant" in argv else None
    print(build(verbose=True, timing="--timing" in argv, variant=var, defines=[a for a in argv if a.startswith("-D")]))
