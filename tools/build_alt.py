#!/usr/bin/env python3
"""Builds an alternate library for A/B timing (NPGX_LIB=<name>): the current
sources with the files given replaced by their text at a git revision.
Usage: tools/build_alt.py TAG REV file [file ...]  -> npge_amd/libnpge_amd_TAG.so"""
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from npge_amd import build as B  # noqa: E402

tag, rev, files = sys.argv[1], sys.argv[2], sys.argv[3:]
tmp = tempfile.mkdtemp()
csrc = os.path.join(tmp, "npge_amd", "csrc")  # common.hpp includes ../../include/npge_amd.h
shutil.copytree(B.CSRC, csrc)
shutil.copytree(os.path.join(ROOT, "include"), os.path.join(tmp, "include"))
for f in files:
    text = subprocess.check_output(["git", "-C", ROOT, "show", "%s:npge_amd/csrc/%s" % (rev, f)])
    open(os.path.join(csrc, f), "wb").write(text)
B.CSRC = csrc
out = B.build(force=True, lib_path=os.path.join(tmp, "lib.so"))
alt = os.path.join(ROOT, "npge_amd", "libnpge_amd_%s.so" % tag)
os.replace(out, alt)
shutil.rmtree(tmp)
print(alt)
