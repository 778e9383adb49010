"""Build the HIP engine (libmtr.so, gfx950) and the synthetic op-log generator in-tree.

Only hipcc/g++ invocations -- no cmake, no JIT caches -- so the built .so files travel to the GPU
box with the repository snapshot.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

ENGINE_SRC = ["mtr_engine.hip"]
ENGINE_DEPS = ["apply.hip.h", "summary.hip.h", "mtr_engine.hip", "apply_caps.hip", "apply_variants.hip"]
CAP_PARTS = 3  # kCapParts in apply.hip.h
VARIANT_PARTS = 5  # kVariantParts in apply.hip.h


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build_engine(force=False, verbose=False, prof=False, variant=None, extra=()):
    """libmtr.so; prof: the phase-timer build (libmtr_prof.so); variant: an experiment build
    libmtr_<variant>.so with extra compiler flags (selected at run time with MTR_LIB)."""
    name = "libmtr_prof.so" if prof else (f"libmtr_{variant}.so" if variant else "libmtr.so")
    out = os.path.join(HERE, name)
    deps = [os.path.join(CSRC, f) for f in ENGINE_DEPS] + [os.path.join(ROOT, "include", h)
                                                           for h in ("mtr.h", "mtr_types.h", "mtr_synth.h", "mtr_digest.h")]
    if force or _stale(out, deps):
        # translation units compiled in parallel (the fixed-capacity kernels in CAP_PARTS parts), then linked
        flags = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wno-unused-result"] + \
            (["-DMTR_PROF"] if prof else []) + list(extra)
        objdir = os.path.join(HERE, "build_prof" if prof else (f"build_{variant}" if variant else "build"))
        os.makedirs(objdir, exist_ok=True)
        units = [(os.path.join(CSRC, f), os.path.join(objdir, f + ".o"), []) for f in ENGINE_SRC]
        units += [(os.path.join(CSRC, "apply_caps.hip"), os.path.join(objdir, f"apply_caps_{q}.o"), [f"-DMTR_CAP_PART={q}"])
                  for q in range(CAP_PARTS)]
        units += [(os.path.join(CSRC, "apply_variants.hip"), os.path.join(objdir, f"apply_variants_{q}.o"),
                   [f"-DMTR_VARIANT_PART={q}"]) for q in range(VARIANT_PARTS)]
        procs = []
        for src, obj, extra in units:
            cmd = flags + extra + ["-c", "-o", obj, src]
            if verbose:
                print(" ".join(cmd))
            procs.append(subprocess.Popen(cmd))
        rcs = [p.wait() for p in procs]
        if any(rcs):
            raise subprocess.CalledProcessError(max(rcs), "hipcc")
        cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out] + [u[1] for u in units]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
    return out


NODE_INCLUDE = "/usr/include/node"


def build_node_addon(force=False, verbose=False):
    """The N-API addon (node/mtr_napi.node) a Node host loads; needs the Node headers, links libmtr.so."""
    src = os.path.join(HERE, "node", "mtr_napi.cc")
    out = os.path.join(HERE, "node", "mtr_napi.node")
    if not os.path.exists(os.path.join(NODE_INCLUDE, "node_api.h")):
        if verbose:
            print("node headers not found: skipping the N-API addon")
        return None
    deps = [src, os.path.join(ROOT, "include", "mtr.h"), os.path.join(HERE, "libmtr.so")]
    if force or _stale(out, deps):
        cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-DNODE_GYP_MODULE_NAME=mtr_napi",
               f"-I{NODE_INCLUDE}", "-o", out, src, f"-L{HERE}", "-lmtr", "-Wl,-rpath,$ORIGIN/.."]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
    return out


def build_all(force=False, verbose=False):
    build_engine(force, verbose)
    build_node_addon(force, verbose)


if __name__ == "__main__":
    if "--prof" in sys.argv:
        build_engine(force="--force" in sys.argv, verbose=True, prof=True)
    elif "--variant" in sys.argv:  # python -m fluidframework_amd.build --variant NAME [flags...]
        i = sys.argv.index("--variant")
        build_engine(force=True, verbose=False, variant=sys.argv[i + 1], extra=sys.argv[i + 2:])
    else:
        build_all(force="--force" in sys.argv, verbose=True)
