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
