"""In-tree build of the scaletorch_amd HIP kernel library for gfx950.

Every ``csrc/*.hip`` file is compiled by ``hipcc --offload-arch=gfx950`` into an
object (pure HIP, no torch headers -> seconds per file); ``csrc/bindings.cpp``
(the TORCH_LIBRARY registrations) is compiled as host C++ against the PyTorch
headers; everything is linked into ``scaletorch_amd/_st_kernels.so``, which
``scaletorch_amd.ops`` loads with ``torch.ops.load_library``.  The ``.so``
lives inside the package so it travels with the repository snapshot to the GPU
box (it is git-ignored but not gpurun-ignored).

Builds are incremental (object newer than its source and ``common.h``) and
run in parallel.  No hipify step, no CUDA sources: the kernels are written for
CDNA4 directly.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
PKG = Path(__file__).resolve().parent
BUILD = ROOT / "build" / "st_kernels"
LIB = PKG / "_st_kernels.so"
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0] or "gfx950"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))

# Per-file flags.  flash_attn: scores never hold NaN by construction (masked
# entries are -inf, never inf - inf), so -fno-honor-nans drops the v_max
# canonicalisation hipcc inserts before every fmaxf on an MFMA result;
# -amdgpu-mfma-vgpr-form keeps compiler-emitted MFMAs in VGPRs (their results
# feed VALU) while the asm accumulate chains own the AGPRs (see mfma_acc).
FILE_FLAGS = {"flash_attn.hip": ["-fno-honor-nans", "-mllvm", "-amdgpu-mfma-vgpr-form"]}


def _hipcc() -> str:
    p = ROCM / "bin" / "hipcc"
    return str(p) if p.exists() else (shutil.which("hipcc") or "hipcc")


def _torch_paths():
    import torch  # noqa: F401
    from torch.utils import cpp_extension as ce

    try:
        inc = ce.include_paths(device_type="cuda")
        libs = ce.library_paths(device_type="cuda")
    except TypeError:  # older signature
        inc = ce.include_paths(cuda=True)
        libs = ce.library_paths(cuda=True)
    return inc, libs


def _stale(obj: Path, deps) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def _run(cmd, verbose: bool):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build step failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return r


def build(verbose: bool = False, jobs: int | None = None, force: bool = False, variant: str | None = None,
          variant_flags: dict | None = None) -> Path:
    """Compile all kernels for ``gfx950`` and link ``_st_kernels.so``; returns its path.

    ``variant``: build an A/B copy into ``build/variants/<variant>.so`` with extra
    per-file flags (``variant_flags = {"flash_attn.hip": [...]}``); load it with
    ``ST_KERNEL_LIB=<path>`` (tools/bench_kernels.py)."""
    global BUILD, LIB
    if variant:
        BUILD = ROOT / "build" / "variants" / variant
        LIB = ROOT / "build" / "variants" / f"{variant}.so"
    BUILD.mkdir(parents=True, exist_ok=True)
    hip_srcs = sorted(CSRC.glob("*.hip"))
    headers = sorted(CSRC.glob("*.h"))
    hipcc = _hipcc()
    common_flags = ["-O3", "-std=c++17", "-fPIC"]
    inc, libdirs = _torch_paths()

    jobs_list = []
    objs = []
    for src in hip_srcs:
        obj = BUILD / (src.stem + ".o")
        objs.append(obj)
        if force or _stale(obj, [src, *headers, Path(__file__)]):
            extra = FILE_FLAGS.get(src.name, []) + (variant_flags or {}).get(src.name, [])
            jobs_list.append([hipcc, f"--offload-arch={ARCH}", *common_flags, *extra, "-c", str(src), "-o",
                              str(obj)])
    # host C++ (torch op registrations, hipBLASLt tuner): g++ against the PyTorch headers
    cxx = shutil.which("g++") or "c++"
    inc_flags = [f"-I{p}" for p in inc] + [f"-I{ROCM / 'include'}"]
    for bsrc in sorted(CSRC.glob("*.cpp")):
        bobj = BUILD / (bsrc.stem + ".o")
        objs.append(bobj)
        if force or _stale(bobj, [bsrc]):
            jobs_list.append(
                [cxx, *common_flags, "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-D_GLIBCXX_USE_CXX11_ABI=1",
                 *inc_flags, "-c", str(bsrc), "-o", str(bobj)]
            )
    n = jobs or min(8, os.cpu_count() or 4)
    if jobs_list:
        with cf.ThreadPoolExecutor(max_workers=n) as ex:
            list(ex.map(lambda c: _run(c, verbose), jobs_list))
    if force or jobs_list or not LIB.exists() or _stale(LIB, objs):
        tmp = LIB.with_suffix(".so.tmp")
        link = [hipcc, "-shared", f"--offload-arch={ARCH}", "-fPIC", *map(str, objs), "-o", str(tmp)]
        for d in libdirs:
            link += [f"-L{d}", f"-Wl,-rpath,{d}"]
        link += ["-lc10", "-lc10_hip", "-ltorch_cpu", "-ltorch_hip", "-ltorch", "-lamdhip64",
                 f"-L{ROCM / 'lib'}", "-lhipblaslt"]
        _run(link, verbose)
        # a library with an unresolved symbol links fine (-shared) and only fails at dlopen:
        # load it once here so a broken build is a build error, not a GPU-box surprise
        chk = subprocess.run([sys.executable, "-c", f"import torch; torch.ops.load_library({str(tmp)!r})"],
                             capture_output=True, text=True)
        if chk.returncode != 0:
            raise RuntimeError(f"built {tmp} does not load:\n{chk.stderr[-2000:]}")
        os.replace(tmp, LIB)
    return LIB


PROBES = "probes"  # the diagnostic library: build/variants/probes.so


def build_probes(verbose: bool = False, force: bool = False) -> Path:
    """The diagnostic library: every kernel file compiled with ``-DST_PROBES``, which adds the
    timing-probe kernels (wrong results by design: DMA / LDS reads / stores / softmax skipped,
    cycle stamps over the output) and their ``ST_*_PROBE`` switches.  The production
    ``_st_kernels.so`` contains none of them; the Python-side probes refuse to run unless this
    library is the loaded one (``ST_KERNEL_LIB=build/variants/probes.so``, ``ops/_lib.py``)."""
    flags = {src.name: ["-DST_PROBES"] for src in CSRC.glob("*.hip")}
    return build(verbose=verbose, force=force, variant=PROBES, variant_flags=flags)


if __name__ == "__main__":
    # python -m scaletorch_amd._build [--force] [-v] [--probes] [--variant NAME file.hip="-flag -flag" ...]
    if "--probes" in sys.argv:
        print(build_probes(verbose="-v" in sys.argv, force="--force" in sys.argv))
        sys.exit(0)
    var, vflags = None, {}
    for a in sys.argv[1:]:
        if a.startswith("--variant="):
            var = a.split("=", 1)[1]
        elif "=" in a and a.split("=", 1)[0].endswith(".hip"):
            f, fl = a.split("=", 1)
            vflags[f] = fl.split()
    p = build(verbose="-v" in sys.argv, force="--force" in sys.argv, variant=var, variant_flags=vflags)
    print(p)
