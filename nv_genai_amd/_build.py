"""In-tree native build for nv_genai_amd.

Two extensions, both built in place so they travel with the repo snapshot to the GPU box:

* ``nv_genai_amd/_C*.so``  — the gfx950 HIP kernels (``csrc/kernels/*.hip``, compiled by
  ``hipcc --offload-arch=gfx950``) plus the PyTorch binding layer (``csrc/bindings.cpp``).
  The kernels themselves include no PyTorch headers; only the binding TU does.
* ``nv_genai_amd/_rt*.so`` — the host-side native runtime (``csrc/runtime/*.cpp``: paged-KV
  block manager, continuous-batching scheduler, BM25 keyword index, token-window splitter),
  plain C++17 + pybind11, so it builds and is unit-tested on a CPU-only machine.

Incremental: an object is rebuilt only when its source (or a header in its directory) is
newer. ``python -m nv_genai_amd._build`` builds everything; ``--clean`` forces a rebuild.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
BUILD = PKG.parent / "build" / "native"
ARCH = os.environ.get("NGA_OFFLOAD_ARCH", "gfx950")
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _hipcc() -> str:
    p = ROCM / "bin" / "hipcc"
    return str(p) if p.exists() else "hipcc"


def _torch_flags():
    import torch  # noqa: F401
    from torch.utils import cpp_extension as ce

    inc = [f"-I{p}" for p in ce.include_paths()]
    libdirs = ce.library_paths()
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    defs = [
        "-D__HIP_PLATFORM_AMD__=1",
        "-DUSE_ROCM=1",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        "-DTORCH_EXTENSION_NAME=_C",
        "-DTORCH_API_INCLUDE_EXTENSION_H",
    ]
    libs = [f"-L{d}" for d in libdirs] + [f"-Wl,-rpath,{d}" for d in libdirs]
    libs += ["-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python"]
    return inc, defs, libs


def _py_inc():
    return [f"-I{sysconfig.get_paths()['include']}"]


def _pybind_inc():
    import pybind11

    return [f"-I{pybind11.get_include()}"]


def _stale(obj: Path, src: Path) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    deps = [src] + list(src.parent.glob("*.h"))
    return any(d.stat().st_mtime > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return r


# MFMA accumulators in VGPRs instead of AGPRs for prefill attention: it rescales its O
# accumulators with VALU ops, and with AGPR accumulators hipcc copied every accumulator
# AGPR->VGPR once per key tile (32 v_accvgpr_read per tile). VGPR form removes the copies
# and lowers the register count (160+44 -> 149, 2 -> 3 waves/SIMD): 735 -> 658 us on 27
# sequences x 1200 tokens. The same flag made decode attention slower (296 -> 335 us at
# 256 x 1400, more resident waves contending for HBM), so it is per file.
PER_FILE_FLAGS = {
    "attention_prefill": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"],
}


def build_kernels(force: bool = False, jobs: int = 8, verbose: bool = False) -> Path:
    """Compile csrc/kernels/*.hip for gfx950 and link the _C extension."""
    out = PKG / f"_C{EXT_SUFFIX}"
    objdir = BUILD / "kernels"
    objdir.mkdir(parents=True, exist_ok=True)
    inc, defs, libs = _torch_flags()
    hip_srcs = sorted((CSRC / "kernels").glob("*.hip"))
    common = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-Wno-unused-result"]
    if os.environ.get("NGA_DIAG_BUILD", "0") != "0":
        # kernel ablation variants (NGA_PV2_ABLATE / NGA_MOE_ABLATE: timings only, results
        # wrong by design) exist only in this build; rebuild with force=True when switching
        common.append("-DNGA_DIAG_ABLATION")
    jobs_list = []
    objs = []
    for s in hip_srcs:
        o = objdir / (s.stem + ".o")
        objs.append(o)
        if force or _stale(o, s):
            jobs_list.append([_hipcc(), *common, *PER_FILE_FLAGS.get(s.stem, []), "-c", str(s), "-o", str(o)])
    bsrc = CSRC / "bindings.cpp"
    bobj = objdir / "bindings.o"
    objs.append(bobj)
    if force or _stale(bobj, bsrc) or any(_stale(bobj, h) for h in (CSRC / "kernels").glob("*.h")):
        jobs_list.append([_hipcc(), "-O2", "-fPIC", "-std=c++17", *defs, *inc, *_py_inc(),
                          "-Wno-unused-result", "-Wno-deprecated-declarations", "-c", str(bsrc),
                          "-o", str(bobj)])
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        for r in ex.map(_run, jobs_list):
            if verbose and r.stderr:
                print(r.stderr, file=sys.stderr)
    if force or jobs_list or not out.exists():
        tmp = out.with_suffix(".tmp.so")
        _run([_hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), "-o",
              str(tmp), *libs])
        os.replace(tmp, out)
    return out


def build_runtime(force: bool = False, jobs: int = 8, out_dir: Path | None = None,
                  extra_flags: list | None = None) -> Path:
    """Compile the host-only native runtime (_rt) with the system C++ compiler.

    ``out_dir``/``extra_flags`` build a variant elsewhere, e.g. the ASan+UBSan build that
    tests/test_runtime_sanitizers.py drives."""
    out = (Path(out_dir) if out_dir else PKG) / f"_rt{EXT_SUFFIX}"
    objdir = (Path(out_dir) / "obj") if out_dir else BUILD / "runtime"
    objdir.mkdir(parents=True, exist_ok=True)
    srcs = sorted((CSRC / "runtime").glob("*.cpp"))
    cxx = os.environ.get("CXX", "g++")
    flags = ["-O2", "-fPIC", "-std=c++17", "-pthread", "-fvisibility=hidden", *_py_inc(), *_pybind_inc()]
    extra = os.environ.get("NGA_RT_CXXFLAGS", "").split() + list(extra_flags or [])
    jobs_list, objs = [], []
    for s in srcs:
        o = objdir / (s.stem + ".o")
        objs.append(o)
        if force or _stale(o, s):
            jobs_list.append([cxx, *flags, *extra, "-c", str(s), "-o", str(o)])
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        list(ex.map(_run, jobs_list))
    if force or jobs_list or not out.exists():
        tmp = out.with_suffix(".tmp.so")
        _run([cxx, "-shared", "-pthread", *map(str, objs), *extra, "-o", str(tmp), "-lrt"])
        os.replace(tmp, out)
    return out


def check_loadable() -> None:
    """Import both extensions in a fresh interpreter: a link that leaves a symbol undefined
    (e.g. a kernel template whose host stub the compiler did not emit) only shows at load
    time, and must fail the build, not the first GPU run."""
    r = subprocess.run([sys.executable, "-c", "import nv_genai_amd._rt, nv_genai_amd._C"],
                       cwd=str(PKG.parent), capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("built extensions do not load:\n" + r.stderr[-2000:])


def build_all(force: bool = False) -> None:
    build_runtime(force=force)
    build_kernels(force=force)
    check_loadable()


if __name__ == "__main__":
    force = "--clean" in sys.argv
    if force and BUILD.exists():
        shutil.rmtree(BUILD)
    build_all(force=force)
    print("built:", sorted(p.name for p in PKG.glob("_*.so")))
