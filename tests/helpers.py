"""Shared test helpers."""
from npge_amd.model import Block, Fragment


def af_blocks_from_result(r, seqs):
    """SoA anchor result -> list of Block (fragments in result order)."""
    blocks = []
    bs = r["block_start"]
    for b in range(len(bs) - 1):
        frs = [Fragment(seqs[int(r["seq"][i])], int(r["min_pos"][i]), int(r["max_pos"][i]),
                        int(r["ori"][i])) for i in range(bs[b], bs[b + 1])]
        blocks.append(Block(frs))
    return blocks


_COMP = {"A": "T", "T": "A", "G": "C", "C": "G", "N": "N"}


def _text(s, start, n, o):
    if o == 1:
        return s[start:start + n]
    return "".join(_COMP[s[start - i]] for i in range(n))


def flank_jobs(blocks, seqs, portion_x1e4=5000, extend_length=100):
    """The right and left flank rows FragmentsExtender aligns for every block
    (FragmentsExtender.cpp:34-119); blocks are oracle-style lists of
    (seq, min, max, ori, row)."""
    jobs = []
    for b in blocks:
        if len(b) < 2:
            continue
        L = len(b[0][4])
        E = max(extend_length, portion_x1e4 * L // 10000)
        for side in (0, 1):
            sh = E
            for (q, mn, mx, ori, _) in b:
                oo = -ori if side else ori
                sh = min(sh, len(seqs[q]) - 1 - mx if oo == 1 else mn)
            if sh <= 0:
                continue
            rows = []
            for (q, mn, mx, ori, _) in b:
                oo = -ori if side else ori
                begin = mn if oo == 1 else mx
                rows.append(_text(seqs[q], begin + oo * (mx - mn + 1), sh, oo))
            jobs.append(rows)
    return jobs


def af_digest(r, used=None):
    """Size-independent fingerprint of an AnchorFinder SoA result: per-array
    sha256 (int64 little-endian) plus the scalar outputs, so full-size runs
    are compared bit-exactly against committed fixtures."""
    import hashlib

    import numpy as np
    d = {k: int(r[k]) for k in ("members", "bits", "hashes", "n_collected", "n_found_frags")}
    d["params"] = [int(x) for x in r["params"]]
    d["n_blocks"] = len(r["block_start"]) - 1
    d["n_fragments"] = len(r["seq"])
    for k in ("block_start", "seq", "min_pos", "max_pos", "ori"):
        a = np.ascontiguousarray(np.asarray(r[k], dtype="<i8"))
        d["sha_" + k] = hashlib.sha256(a.tobytes()).hexdigest()
    if used is not None:
        a = np.ascontiguousarray(np.asarray(used, dtype="<u8"))
        d["n_used"] = len(a)
        d["sha_used"] = hashlib.sha256(a.tobytes()).hexdigest()
    return d


def blocks_digest(blocks):
    """Order-free fingerprint of a block set given as lists of
    (seq, min, max, ori, row) tuples (BlockSetEngine.blocks() and
    BlockSetOracle.blocks() share that form)."""
    import hashlib
    canon = sorted(tuple(sorted((int(q), int(a), int(b), int(o), r) for (q, a, b, o, r) in blk))
                   for blk in blocks)
    return {"n_blocks": len(canon), "n_fragments": sum(len(b) for b in canon),
            "sha_blocks": hashlib.sha256(repr(canon).encode()).hexdigest()}


def oracle_anchor_blocks(r):
    """(oracle.anchor_blocks)"""
    from oracle import oracle as orc
    return orc.anchor_blocks(r)


def consensus_order(b):
    """(oracle.consensus_order: the pinned ConSeq block order)"""
    from oracle import oracle as orc
    return orc.consensus_order(b)


def oracle_anchor_loop(o, workers=1):
    """AnchorLoopFast over the oracle's processors (oracle.anchor_loop_fast,
    lua_lib.lua:741-758)."""
    from oracle import oracle as orc
    return orc.anchor_loop_fast(o, workers)


_GOLD = 0x9E3779B97F4A7C15
_M64 = (1 << 64) - 1


def _sm(x):
    """splitmix64 output of x + golden ratio, vectorised over uint64 arrays."""
    import numpy as np
    with np.errstate(over="ignore"):
        z = np.asarray(x, dtype=np.uint64) + np.uint64(_GOLD)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def rows_digest(blocks):
    """npgx_blockset_rows_digest restated (include/npge_amd.h): blocks are lists
    of (seq, min, max, ori, row); every row bound to its fragment's key,
    summed mod 2^64, independent of the block order."""
    import numpy as np
    total = 0
    for b in blocks:
        for (q, mn, mx, ori, row) in b:
            if row is None:
                continue
            key = int(_sm(int(_sm(int(_sm(2 * q + (1 if ori > 0 else 0))) + mn) & _M64) + mx) & _M64)
            r = np.frombuffer(row.encode(), dtype=np.uint8).astype(np.uint64)
            c = np.arange(len(r), dtype=np.uint64)
            with np.errstate(over="ignore"):
                cells = _sm(np.uint64(key) ^ ((c << np.uint64(8)) | r))
                total = (total + int(_sm((key + len(r)) & _M64)) + int(cells.sum(dtype=np.uint64))) & _M64
    return total
