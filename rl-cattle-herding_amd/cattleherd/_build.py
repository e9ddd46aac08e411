"""Compile libcattleherd.so (HIP kernels + C ABI) in-tree for gfx950.

The .so is written next to this file so it travels to the GPU box with the repo snapshot.
"""
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build")
LIB = os.path.join(PKG, "libcattleherd.so")
SOURCES = ["ch_kernels.hip", "ch_step.hip", "ch_step_multi.hip", "ch_policy.hip", "ch_aux.hip", "ch_api.cpp"]
# per-source flags: ch_step_multi.hip's step loop keeps k_step2's register allocation only with machine LICM off
# (ch_step_multi.hip header)
SOURCE_FLAGS = {"ch_step_multi.hip": ["-mllvm", "-disable-machine-licm"]}
HEADERS = ["ch_device.h", "ch_internal.h", "ch_common.h", "ch_spawn_table.inc", "ch_mlp2_dev.h", "ch_rollout_dev.h"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("CH_OFFLOAD_ARCH", "gfx950")
# fp-contract off: the fp64 path keeps the reference's rounding (no fused multiply-adds), so it
# reproduces the CPU oracle to the last few ulps.
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", f"--offload-arch={ARCH}",
         "-I" + os.path.join(os.path.dirname(ROOT), "include")]


def _stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + \
        [os.path.join(os.path.dirname(ROOT), "include", "cattleherd.h"), __file__]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=False, extra_flags=(), out=None):
    lib_out = out or LIB
    if not force and out is None and not _stale():
        return LIB
    os.makedirs(BUILD, exist_ok=True)
    objs, procs = [], []
    # the translation units compile in parallel (ch_step.hip's instantiations dominate the build)
    for src in SOURCES:
        obj = os.path.join(BUILD, src + ("".join(extra_flags).replace("-", "_") if extra_flags else "") + ".o")
        cmd = [HIPCC, *FLAGS, *SOURCE_FLAGS.get(src, []), *extra_flags, "-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((cmd, subprocess.Popen(cmd)))
        objs.append(obj)
    failed = [cmd for cmd, p in procs if p.wait() != 0]
    if failed:
        raise subprocess.CalledProcessError(1, failed[0])
    tmp = lib_out + ".tmp"
    cmd = [HIPCC, *FLAGS, "-shared", *objs, "-o", tmp]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, lib_out)
    return lib_out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
