"""Flags vector stores whose 64-bit address registers overlap their data
registers in the gfx950 device code of npge_amd/csrc/*.hip.

Round 5 found one such store from the ROCm 7.2 compiler: in
k_pass_fill<PlanPass> (elf_device.inc) the second side's copy of the flank-row
loop wrote each row's address over the row's start position
(`global_store_dwordx4 v[2:3], v[2:5]`).  The source now pins the loaded values
in registers before the select; this lint re-checks every kernel after changes.
Stores addressed by an SGPR base with a VGPR offset (`global_store_dword v1,
v1, s[0:1]`: zero stored at offset zero) are not flagged.

    python tools/isa_store_lint.py [source.hip ...]
"""
import glob
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
PAT = re.compile(r"(global|flat|buffer)_store_\w+\s+v\[(\d+):(\d+)\],\s+v(?:\[(\d+):(\d+)\]|(\d+))")


def lint(src, out_dir):
    asm = os.path.join(out_dir, os.path.basename(src) + ".s")
    subprocess.run(["hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-munsafe-fp-atomics",
                    "--cuda-device-only", "-S", "-I", os.path.join(REPO, "include"), src, "-o", asm],
                   check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    hits, fn = [], None
    with open(asm) as f:
        for ln, line in enumerate(f, 1):
            if line[:1] not in ("", " ", "\t", ".", ";") and line.rstrip().endswith(":"):
                fn = line.split(":")[0]
            m = PAT.search(line)
            if not m:
                continue
            a0, a1 = int(m.group(2)), int(m.group(3))
            d0, d1 = (int(m.group(4)), int(m.group(5))) if m.group(4) else (int(m.group(6)),) * 2
            if not (d1 < a0 or d0 > a1):
                hits.append((fn, ln, line.strip()))
    return hits


def lint_all(srcs=None, jobs=8):
    """{source basename: [(function, asm line, store)]} over the sources
    (default: every npge_amd/csrc/*.hip), compiled in parallel."""
    from concurrent.futures import ThreadPoolExecutor
    srcs = srcs or sorted(glob.glob(os.path.join(REPO, "npge_amd", "csrc", "*.hip")))
    with tempfile.TemporaryDirectory() as d:
        with ThreadPoolExecutor(max(1, jobs)) as ex:
            res = list(ex.map(lambda s: lint(s, d), srcs))
    return {os.path.basename(s): h for s, h in zip(srcs, res)}


def main():
    bad = 0
    for name, hits in lint_all(sys.argv[1:] or None).items():
        print("%s: %d overlapping stores" % (name, len(hits)))
        for h in hits:
            print("   %s (line %d): %s" % h)
        bad += len(hits)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
