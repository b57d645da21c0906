"""In-tree native build of ``distributed_pytorch_hpc_amd/_C.so`` (gfx950 only).

Device code (``csrc/*.hip``) is compiled by ``hipcc --offload-arch=gfx950`` WITHOUT any torch header,
the dispatcher glue (``csrc/torch_ops.cpp``) by ``g++`` against the torch headers, and both are linked
into one shared object that ``torch.ops.load_library`` loads.  No hipify, no cpp_extension JIT cache:
the ``.so`` lives next to the package so it travels with the repo snapshot to the GPU box.

The ninja file makes rebuilds incremental (only edited kernels recompile).

Usage:  python -m distributed_pytorch_hpc_amd.csrc.build [--jobs N] [--verbose]
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
BUILD_DIR = os.path.join(PKG, "..", "build", "native")
OUT = os.path.join(PKG, "_C.so")
ARCH = os.environ.get("DPH_OFFLOAD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
# attention.hip (the forward): no NaN semantics needed (masks are -inf, never NaN), and IEEE mode off so fmaxf on MFMA
# results is a bare v_max / v_max3 instead of a canonicalising v_max per operand first (the row max of every score
# tile): forward 814 -> 836 TFLOP/s.  attention_bwd.hip has no row max and is built WITHOUT them: under these flags
# the dK/dV kernel's register allocation spills 80 B at 256 VGPRs (the reloads drain the in-flight Q / dO prefetch),
# backward 702 -> 655 TFLOP/s (profiles/r5/attn_split/).
PER_FILE_HIP_FLAGS = {"attention.hip": ["-fno-honor-nans", "-mno-amdgpu-ieee"]}


def _torch_paths():
    import torch

    root = os.path.dirname(torch.__file__)
    inc = [os.path.join(root, "include"), os.path.join(root, "include", "torch", "csrc", "api", "include")]
    lib = os.path.join(root, "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def sources():
    hip = sorted(f for f in os.listdir(HERE) if f.endswith(".hip"))
    cpp = sorted(f for f in os.listdir(HERE) if f.endswith(".cpp"))
    return hip, cpp


def write_ninja(build_dir: str, verbose_asm: bool = False) -> str:
    inc, lib, abi = _torch_paths()
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    hip_flags = [
        f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=fast", "-munsafe-fp-atomics",
        f"-I{HERE}", "-Wno-unused-result",
    ]
    if verbose_asm:
        hip_flags.append("-Rpass-analysis=kernel-resource-usage")
    cxx_flags = [
        "-O2", "-std=c++17", "-fPIC", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-D__HIP_PLATFORM_AMD__=1",
        "-DUSE_ROCM=1", "-Wno-deprecated-declarations", f"-I{HERE}", f"-I{ROCM}/include",
        f"-I{sysconfig.get_paths()['include']}",
    ] + [f"-I{p}" for p in inc]
    ldflags = [
        "-shared", f"-L{lib}", f"-Wl,-rpath,{lib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
        "-lamdhip64",
    ]
    hip, cpp = sources()
    lines = [
        "ninja_required_version = 1.3",
        f"hipcc = {hipcc}",
        "cxx = g++",
        "hipflags = " + " ".join(hip_flags),
        "cxxflags = " + " ".join(cxx_flags),
        "ldflags = " + " ".join(ldflags),
        "rule hipcc",
        "  command = $hipcc $hipflags -MD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = HIPCC $in",
        "rule cxx",
        "  command = $cxx $cxxflags -MD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = CXX $in",
        "rule link",
        "  command = $cxx $in -o $out $ldflags",
        "  description = LINK $out",
    ]
    objs = []
    for f in hip:
        o = os.path.join(build_dir, f + ".o")
        lines.append(f"build {o}: hipcc {os.path.join(HERE, f)}")
        if f in PER_FILE_HIP_FLAGS:
            lines.append("  hipflags = $hipflags " + " ".join(PER_FILE_HIP_FLAGS[f]))
        objs.append(o)
    for f in cpp:
        o = os.path.join(build_dir, f + ".o")
        lines.append(f"build {o}: cxx {os.path.join(HERE, f)}")
        objs.append(o)
    lines.append(f"build {OUT}: link " + " ".join(objs))
    lines.append(f"default {OUT}")
    path = os.path.join(build_dir, "build.ninja")
    with open(path, "w") as fh:
        fh.write("\n".join(lines) + "\n")
    return path


def build(jobs: int | None = None, verbose: bool = False, resource_usage: bool = False) -> str:
    build_dir = os.path.abspath(BUILD_DIR)
    os.makedirs(build_dir, exist_ok=True)
    ninja_file = write_ninja(build_dir, resource_usage)
    ninja = shutil.which("ninja")
    if ninja is None:
        raise RuntimeError("ninja not found")
    jobs = jobs or min(8, os.cpu_count() or 4)
    if os.environ.get("DPH_BUILD_CLEAN", "0") == "1":   # force every object to recompile (a from-scratch build check)
        subprocess.run([ninja, "-f", ninja_file, "-t", "clean"], check=True, cwd=build_dir, stdout=subprocess.DEVNULL)
    cmd = [ninja, "-f", ninja_file, "-j", str(jobs)]
    if verbose:
        cmd.append("-v")
    res = subprocess.run(cmd, cwd=build_dir, stdout=subprocess.PIPE, text=True)
    sys.stdout.write(res.stdout)   # ninja's log, compiler diagnostics included
    if res.returncode != 0:
        raise subprocess.CalledProcessError(res.returncode, cmd)
    # what this call actually compiled: ninja prints one "[i/n] ..." line per edge it ran, nothing when up to date
    ran = [ln for ln in res.stdout.splitlines() if ln.startswith("[")]
    n_hip = sum(1 for f in os.listdir(HERE) if f.endswith(".hip"))
    n_cpp = sum(1 for f in os.listdir(HERE) if f.endswith(".cpp"))
    compiled = sum(1 for ln in ran if "HIPCC" in ln or "CXX" in ln)
    print(f"[build] {ARCH}: {compiled} of {n_hip + n_cpp} sources ({n_hip} .hip + {n_cpp} .cpp) compiled this call"
          f"{' (rest up to date)' if compiled < n_hip + n_cpp else ''}; linked: {any('LINK' in ln for ln in ran)}")
    return OUT


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=None)
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--resource-usage", action="store_true", help="print VGPR/SGPR/LDS per kernel")
    args = ap.parse_args(argv)
    out = build(args.jobs, args.verbose, args.resource_usage)
    print(out)


if __name__ == "__main__":
    sys.exit(main())
