"""Generates tests/golden/glibc_rand.json from this machine's glibc srand/rand
(the generator behind BloomFilter::set_hashes, BloomFilter.cpp:55-63), to pin
the oracle's and the product's restatement of glibc TYPE_3 rand()."""
import ctypes
import json
import os

libc = ctypes.CDLL("libc.so.6")
out = {}
for seed in [0, 1, 2, 7, 42, 12345, 987654321, 2**31 - 1, 2**32 - 1]:
    libc.srand(ctypes.c_uint(seed))
    out[str(seed)] = [libc.rand() for _ in range(40)]
with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "glibc_rand.json"), "w") as f:
    json.dump(out, f, indent=0)
