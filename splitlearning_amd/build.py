"""In-tree native build: compile the gfx950 HIP kernels + bindings into
`splitlearning_amd/_C<ext>.so` with hipcc (no hipify, no JIT cache).

    python -m splitlearning_amd.build          # incremental
    python -m splitlearning_amd.build --force  # rebuild everything

Objects go to `splitlearning_amd/build/` (git-ignored); the `.so` lands next to
this file so `gpurun` snapshots carry it to the GPU box.  Cross-compiles fine on
a host without a GPU.
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "build")
ARCH = os.environ.get("SL_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

KERNEL_SOURCES = ["conv.hip", "linear.hip", "loss.hip", "fused.hip", "gemm.hip", "ipc_ar.hip", "ipc_p2p.hip", "resident.hip", "hybrid.hip", "vanilla.hip", "handoff.hip", "ushape.hip"]
BINDING_SOURCES = ["bindings.cpp", "comm.cpp", "engine.cpp", "split.cpp", "resident_exec.cpp", "hybrid_exec.cpp", "vanilla_exec.cpp", "ushape_exec.cpp"]


def so_path() -> str:
    return os.path.join(HERE, "_C" + sysconfig.get_config_var("EXT_SUFFIX"))


def _torch_flags():
    import torch
    from torch.utils import cpp_extension as ce
    inc = ce.include_paths()
    tlib = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cflags = [f"-I{p}" for p in inc] + [f"-I{sysconfig.get_paths()['include']}",
                                        f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
                                        "-DTORCH_API_INCLUDE_EXTENSION_H",
                                        "-DTORCH_EXTENSION_NAME=_C", "-DUSE_ROCM=1"]
    ldflags = [f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
               "-ltorch_python", "-lamdhip64", "-lrccl", f"-Wl,-rpath,{tlib}"]
    return cflags, ldflags


BASE = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-D__HIP_PLATFORM_AMD__=1",
        "-Wno-unused-result", "-Wno-deprecated-declarations"]


def _stale(src: str, obj: str, deps: list[str]) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in [src] + deps)


def _compile(src: str, extra: list[str], force: bool) -> str:
    obj = os.path.join(OBJ, os.path.basename(src) + ".o")
    deps = [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".h")]
    if force or _stale(src, obj, deps):
        cmd = [HIPCC] + BASE + ["-x", "hip", "-c", src, "-o", obj] + extra
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{' '.join(cmd)}\n{r.stderr[-6000:]}")
    return obj


def build(force: bool = False, verbose: bool = True) -> str:
    os.makedirs(OBJ, exist_ok=True)
    cflags, ldflags = _torch_flags()
    jobs = [(os.path.join(CSRC, s), []) for s in KERNEL_SOURCES]
    jobs += [(os.path.join(CSRC, s), cflags) for s in BINDING_SOURCES]
    with ThreadPoolExecutor(max_workers=min(8, len(jobs))) as ex:
        objs = list(ex.map(lambda j: _compile(j[0], j[1], force), jobs))
    out = so_path()
    if force or not os.path.exists(out) or any(os.path.getmtime(o) > os.path.getmtime(out) for o in objs):
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", out] + objs + ldflags
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{r.stderr[-6000:]}")
    if verbose:
        print(f"[splitlearning_amd.build] {out}")
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args(argv)
    build(force=a.force)


if __name__ == "__main__":
    sys.exit(main())
