"""Builds the in-tree HIP library npge_amd/libnpge_amd.so for gfx950 with hipcc.

hipcc cross-compiles without a GPU, so this runs in the CPU container; the .so
travels to the GPU box with the repo snapshot.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libnpge_amd.so")
# diagnostic variant with per-phase cycle counters in the aligner kernel
# (loaded by _capi when NPGX_PROFILE=1)
LIB_PROF = os.path.join(HERE, "libnpge_amd_prof.so")
SOURCES = ["seqset.hip", "anchor_finder.hip", "similar_aligner.hip", "block_build.hip",
           "general_aligner.hip", "wide_aligner.hip", "comm_rccl.hip", "host_sampler.cpp"]
HEADERS = ["common.hpp", "sa_device.hpp", "log_score.inc", "elf_device.inc"]
ARCH = os.environ.get("NPGX_OFFLOAD_ARCH", "gfx950")


def _stale(lib=LIB):
    if not os.path.exists(lib):
        return True
    t = os.path.getmtime(lib)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    deps.append(os.path.join(os.path.dirname(HERE), "include", "npge_amd.h"))
    return any(os.path.exists(d) and os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=False, profile=False, lib_path=None, defines=()):
    """defines: extra -D flags for an A/B variant (e.g. ("SA_FAST_ROWS=1",))."""
    lib = lib_path or (LIB_PROF if profile else LIB)
    if not force and not _stale(lib):
        return lib
    objs = []
    procs = []
    for src in [x for x in SOURCES if os.path.exists(os.path.join(CSRC, x))]:
        stem, ext = os.path.splitext(src)
        obj = os.path.join(CSRC, stem + ("_prof.o" if profile else ".o"))
        if ext == ".cpp":  # host-only helpers
            cmd = ["g++", "-c", "-O2", "-std=c++17", "-fPIC", "-o", obj, os.path.join(CSRC, src)]
        else:
            cmd = ["hipcc", "-c", "-O3", "-std=c++17", "-fPIC", "--offload-arch=" + ARCH,
                   "-munsafe-fp-atomics", "-Wno-unused-result", "-I", os.path.join(os.path.dirname(HERE), "include"),
                   "-o", obj, os.path.join(CSRC, src)] + (["-DNPGX_SA_PROFILE=1"] if profile else []) + \
                  ["-D" + d for d in defines]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((src, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
        objs.append(obj)
    for src, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            raise RuntimeError("hipcc failed on %s:\n%s" % (src, out.decode(errors="replace")))
    tmp = lib + ".tmp"
    cmd = ["hipcc", "-shared", "-fPIC", "--offload-arch=" + ARCH, "-o", tmp] + objs + ["-lrccl"]
    subprocess.check_call(cmd)
    os.replace(tmp, lib)
    for o in objs:
        os.remove(o)
    return lib


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True, profile="--profile" in sys.argv))
