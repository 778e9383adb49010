"""Build the HIP engine (libmtr.so, gfx950) and the synthetic op-log generator in-tree.

Only hipcc/g++ invocations -- no cmake, no JIT caches -- so the built .so files travel to the GPU
box with the repository snapshot.
"""
from __future__ import annotations

import json
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

ENGINE_SRC = ["mtr_engine.hip"]
ENGINE_DEPS = ["apply.hip.h", "summary.hip.h", "mtr_engine.hip", "apply_caps.hip", "apply_variants.hip"]
CAP_PARTS = 3  # kCapParts in apply.hip.h
VARIANT_PARTS = 16  # kVariantParts in apply.hip.h


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


_REMARK = re.compile(r"remark: +([A-Za-z][A-Za-z /\[\]]*?): (.*?) \[-Rpass-analysis=kernel-resource-usage\]")


def kernel_resources(stderr_texts):
    """Per kernel (mangled name): the compiler's resource-usage remarks (VGPRs, ScratchSize, spills, occupancy)."""
    res, cur = {}, None
    for text in stderr_texts:
        for line in text.splitlines():
            m = _REMARK.search(line)
            if not m:
                continue
            k, v = m.group(1).strip(), m.group(2).strip()
            if k == "Function Name":
                cur = res.setdefault(v, {})
            elif cur is not None:
                cur[k] = int(v) if v.lstrip("-").isdigit() else v
    return res


# No apply kernel may spill VGPRs (apply_kernel / apply_pair_kernel / apply_pair2_kernel, LDS- and HBM-resident), and
# the lean HBM-resident one (CAP = -1: C5's kernel) must use no scratch at all.  A round-3 build whose lean HBM kernel
# spilled produced wrong views; the main build refuses one.  (The X / delta / record-mode
# kernels keep some scratch that is no spill: the call frames of their out-of-line rare paths -- regenerate, normalize,
# props_apply_serial, props_restore -- whose by-reference document structs live on the stack, and a few dynamically
# indexed private arrays)
_APPLY_KERNELS = re.compile(r"^_ZN3mtr(12apply_kernel|17apply_pair_kernel|18apply_pair2_kernel)I")
_HBM_LEAN = re.compile(r"^_ZN3mtr12apply_kernelILb1ELin1E")


def check_no_scratch(res, strict=True):
    bad = {}
    for k, v in res.items():
        if not _APPLY_KERNELS.match(k):
            continue
        scratch, vspill = v.get("ScratchSize [bytes/lane]", 0), v.get("VGPRs Spill", 0)
        if vspill or (_HBM_LEAN.match(k) and scratch):
            bad[k] = (scratch, vspill)
    if bad:
        msg = "apply kernels spill VGPRs: " + ", ".join(
            f"{k} (scratch {a} B/lane, {b} VGPRs spilled)" for k, (a, b) in sorted(bad.items()))
        if strict:
            raise RuntimeError(msg)
        print("warning: " + msg, file=sys.stderr)
    return bad


def build_engine(force=False, verbose=False, prof=False, variant=None, extra=()):
    """libmtr.so; prof: the phase-timer build (libmtr_prof.so); variant: an experiment build
    libmtr_<variant>.so with extra compiler flags (selected at run time with MTR_LIB)."""
    name = "libmtr_prof.so" if prof else (f"libmtr_{variant}.so" if variant else "libmtr.so")
    out = os.path.join(HERE, name)
    deps = [os.path.join(CSRC, f) for f in ENGINE_DEPS] + [os.path.join(ROOT, "include", h)
                                                           for h in ("mtr.h", "mtr_types.h", "mtr_synth.h", "mtr_digest.h")]
    if True:  # (each translation unit is checked against its sources below; the library against its objects)
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
        hdrs = [d for d in deps if d.endswith(".h")]
        flag_file = os.path.join(objdir, "flags.txt")
        same_flags = os.path.exists(flag_file) and open(flag_file).read() == " ".join(flags)
        reuse = variant and os.environ.get("MTR_REUSE_VARIANTS") == "1"
        # (development: MTR_ONLY=apply_variants_3,mtr_engine recompiles just the units named, keeping the other
        # objects as they are -- for an edit whose effect is confined to those units' kernels)
        only = [x for x in os.environ.get("MTR_ONLY", "").split(",") if x]
        for src, obj, extra in units:
            if only and not any(x in os.path.basename(obj) for x in only):
                main_obj = os.path.join(HERE, "build", os.path.basename(obj))
                if not os.path.exists(obj) and os.path.exists(main_obj):  # (a variant: the main build's object)
                    import shutil

                    shutil.copy(main_obj, obj)
                if os.path.exists(obj):
                    continue
            if same_flags and not force and not _stale(obj, [src] + hdrs):
                continue  # (per translation unit: an edit of one .hip recompiles that unit only)
            if reuse and "apply_variants" in obj:  # (a C3 experiment: the runtime-layout kernels from the main build)
                import shutil

                shutil.copy(os.path.join(HERE, "build", os.path.basename(obj)), obj)
                continue
            cmd = flags + extra + ["-Rpass-analysis=kernel-resource-usage", "-c", "-o", obj, src]
            if verbose:
                print(" ".join(cmd))
            procs.append(subprocess.Popen(cmd, stderr=subprocess.PIPE, text=True))
        if not procs and not _stale(out, [u[1] for u in units]):
            return out
        outs = [p.communicate()[1] for p in procs]
        rcs = [p.returncode for p in procs]
        if any(rcs):
            for o in outs:
                sys.stderr.write("\n".join(l for l in o.splitlines() if "kernel-resource-usage" not in l) + "\n")
            raise subprocess.CalledProcessError(max(rcs), "hipcc")
        rpath = os.path.join(objdir, "kernel_resources.json")
        res = json.load(open(rpath)) if os.path.exists(rpath) else {}
        res.update(kernel_resources(outs))
        with open(rpath, "w") as f:
            json.dump(res, f, indent=1, sort_keys=True)
        with open(flag_file, "w") as f:
            f.write(" ".join(flags))
        check_no_scratch(res, strict=not (variant or prof) or os.environ.get("MTR_REQUIRE_NO_SCRATCH") == "1")
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
